# round 6: hipIpc same-device import sweep (bench/ipc_import_repro): importer holds X GiB,
# exporter exports Y GiB in <= 32 GiB segments; points in ascending X + Y; the sweep STOPS at
# the first point that times out or fails (no further GPU step after a hang)
set -u
O=gpurun_out/s9ipc; mkdir -p $O
B=./bench/ipc_import_repro
POINTS=${POINTS:-"0:32 0:96 64:32 64:96 128:32 96:96 128:96 192:32 160:96 128:128"}
for pt in $POINTS; do
  X=${pt%%:*}; Y=${pt##*:}
  D=$(mktemp -d /tmp/ipcrepro.XXXX)
  timeout -k 5 90 $B export $Y 32 $D > $O/x${X}_y${Y}.export.log 2>&1 &
  EP=$!
  timeout -k 5 60 $B import $X $D > $O/x${X}_y${Y}.import.log 2>&1
  IRC=$?
  wait $EP; ERC=$?
  rm -rf $D
  echo "X=$X Y=$Y import_rc=$IRC export_rc=$ERC"
  tail -1 $O/x${X}_y${Y}.import.log
  if [ $IRC -ne 0 ] || [ $ERC -ne 0 ]; then echo "stop at X=$X Y=$Y"; exit 1; fi
done
echo "sweep done"

set -u
O=gpurun_out/r4r; mkdir -p $O
timeout -k 10 120 ./tools/probes/stream_probe > $O/stream.log 2>&1; echo "stream rc=$?"

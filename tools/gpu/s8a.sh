# round 6, first GPU check: IPC collectives + TP/PD processes (error-word probe, kv id guard),
# kv kernels, engine, smoke, baseline bench
set -u
O=gpurun_out/s8a; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
P="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
run ingress 120 ./tools/probes/ingress_probe &&
run t_kv 300 $P tests/test_kernels_gpu.py -k "kv" &&
run t_car 300 $P tests/test_custom_allreduce_gpu.py &&
run t_tp 400 $P tests/test_tp_gpu.py &&
run t_pd 300 $P tests/test_pd_gpu.py &&
run t_engine 400 $P tests/test_engine_gpu.py &&
run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" &&
run bench 400 python -u bench.py &&
echo done

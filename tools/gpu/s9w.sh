# round 6: prefill attention as one flat longest-first (tile, kv head) grid (the scheduler sorts
# the tile map by causal work; AKAP_TILE_SORT=0 keeps map order): attention tests, micro sorted
# vs unsorted map, headline A/B
set -u
O=gpurun_out/s9w; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run t_attn 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "attention or prefill" &&
run ap_sorted 300 python -u tools/attn_prefill_probe.py &&
PROBE_UNSORTED=1 run ap_unsorted 300 python -u tools/attn_prefill_probe.py &&
run b1a 400 python -u bench.py &&
AKAP_TILE_SORT=0 run b0a 400 python -u bench.py &&
run b1b 400 python -u bench.py &&
AKAP_TILE_SORT=0 run b0b 400 python -u bench.py &&
echo done

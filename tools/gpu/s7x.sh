# same-box A/B of the prefill q prep on Llama-3-8B monolithic (TTFT)
set -u
O=gpurun_out/s7x; mkdir -p $O
export TMPDIR=/tmp
run() { local n=$1 tm=$2; shift 2; timeout -k 10 $tm "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run l1 500 python -u bench.py --model llama-3-8b --steps 2 &&
AKAP_PREFILL_QPREP=0 run l0 500 python -u bench.py --model llama-3-8b --steps 2 &&
run l1b 500 python -u bench.py --model llama-3-8b --steps 2 &&
AKAP_PREFILL_QPREP=0 run l0b 500 python -u bench.py --model llama-3-8b --steps 2 &&
echo done

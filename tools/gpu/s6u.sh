# prefill attention timing at the headline prefill chunk (+ Llama-3-8B heads, long prompts)
set -u
O=gpurun_out/s6u; mkdir -p $O
export TMPDIR=/tmp
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run attn 200 python -u tools/attn_prefill_probe.py &&
echo done

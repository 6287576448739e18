# decode-step anatomy (op-class knockouts in the captured step) on the final round-4 tree
set -u
O=gpurun_out/r5k; mkdir -p $O
run() { n=$1; t=$2; shift 2; timeout -k 10 $t "$@" > $O/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ]; }
run qwen3 300 python -u bench/decode_anatomy.py --model qwen3-0.6b --B 256 --ctx 640 &&
run llama8b 300 python -u bench/decode_anatomy.py --model llama-3-8b --B 256 --ctx 640 &&
echo done

# round 3, batch 9: full GPU suite + smoke (as the driver runs them), then the CU-mask probe
set -o pipefail
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputests_r3e.log 2>&1 && \
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r3e.log 2>&1 && \
timeout -k 10 300 python -u tools/cumask_probe.py > gpurun_out/cumask.log 2>&1

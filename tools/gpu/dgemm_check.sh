OVERLAP_GROUP=7 timeout -k 10 200 python -X faulthandler -u bench/overlap_micro.py > gpurun_out/overlap_g7.log 2>&1 && \
OVERLAP_GROUP=4 timeout -k 10 200 python -X faulthandler -u bench/overlap_micro.py > gpurun_out/overlap_g4.log 2>&1

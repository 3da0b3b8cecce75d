export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_list.py -x -v --timeout 200 --timeout-method thread -k "deal or two_waves or c2_trajectory" > gpurun_out/r03c_deal_tests.log 2>&1 || { tail -30 gpurun_out/r03c_deal_tests.log; exit 1; }
tail -3 gpurun_out/r03c_deal_tests.log
bash tools/deal_sweep.sh r03c_deal "rr 001 00101 0010101" "rr 0120123 012012013 0120120123"

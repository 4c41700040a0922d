export TMPDIR=/tmp; O=gpurun_out/r05av; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1 &&
timeout -k 10 300 python bench.py > $O/bench.log 2>&1; rc=$?; tail -n 3 $O/pytest_gpu.log; tail -c 600 $O/bench.log; exit $rc

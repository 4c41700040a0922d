export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 2 --warmup 1 > gpurun_out/bench_full.log 2>&1; echo bench=$?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_mk -o run --output-format csv -- python bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/prof_mk.log 2>&1; echo prof=$?
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_fetch.log 2>&1; echo fetch=$?
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_write.log 2>&1; echo write=$?

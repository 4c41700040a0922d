#!/bin/bash
# One parametrised runner for every GPU-box job (run through gpurun from the repo root):
#   bash tools/gpu_task.sh TASK [TASK ...]     tasks run in order; the first failure ends the call
# Tasks:
#   tests            python -m pytest tests -m gpu (log: gpurun_out/$TAG/pytest_gpu.log)
#   tests:EXPR       the same with -k EXPR
#   smoke            __graft_entry__.smoke()
#   bench            python bench.py (headline line, cpu_baseline included)
#   rehearse[:N]     the N-rank bench path (default 2) on this one GPU: torchrun, every rank on GPU 0
#                    (RT_BENCH_DEVICE=0), 1 step; its frame_sha1 must equal N = 1's
#   trace            rocprofv3 --kernel-trace --stats of `python bench.py --no-cpu-baseline`
#   ktrace:SCRIPT[:ARGS]  rocprofv3 --kernel-trace --stats of `python SCRIPT ARGS` (":" separates args);
#                    per-kernel totals -> $OUT/ktrace_<n>/run_kernel_stats.csv
#   benchpmc         counter passes over `bench.py --steps 1 --warmup 0`: HBM bytes -> $OUT/pmc_traffic.json,
#                    VALU mix + clock -> $OUT/pmc_valu.json (bench.py roofline.traffic / .compute)
#   configs          tools/configs_bench.py (every BASELINE config, one GPU)
#   pmc:SCENE:W:H:SPP[:mis]   counter passes on one megakernel render (tools/prof_render.py):
#                    HBM traffic (FETCH_SIZE / WRITE_SIZE), L2 hit rate (TCC_HIT / TCC_MISS), clock
#                    (GRBM_GUI_ACTIVE) and the SQ instruction mix, each pass a run of its own
#   pmcw:SCENE:W:H:SPP[:mis]  the wait / latency breakdown of one render (SQ_WAIT_*, SQ_ACTIVE_INST_*,
#                    SQ_INST_LEVEL_* over SQ_INSTS_*: mean in-flight latency per memory class)
#   py:SCRIPT[:ARGS] python SCRIPT ARGS (":" separates args), e.g. py:tools/configs_bench.py:--quick
#   env:VAR=VAL[,VAR=VAL]  export for the following tasks (A/B of the RT_* switches)
#   avail            rocprofv3 --list-avail -> $OUT/avail.txt
#   dbgbuild         build the diagnostic library lib/variants/dbg.so (better: build it here and ship it)
# Env: TAG (output subdirectory, default "run"), BENCH_ARGS (extra bench.py arguments).
export TMPDIR=/tmp
TAG=${TAG:-run}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
KT=0

fail() { echo "FAIL: $1"; [ -f "$2" ] && tail -30 "$2"; exit 1; }

# SQ passes: at most 8 SQ counters each
SQ1="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU"
SQ2="SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_THREAD_CYCLES_VALU SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_TRANS_F64"
# wait / latency breakdown (pmcw): where waves spend the cycles they do not issue
SQW1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM"
SQW2="SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_INST_LEVEL_SMEM SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_ANY"
SQ3="SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_LDS"

pmc_pass() {  # name counters... -- command
    local name=$1; shift
    local ctr=()
    while [ "$1" != "--" ]; do ctr+=("$1"); shift; done
    shift
    timeout -s KILL 120 rocprofv3 --pmc "${ctr[@]}" -d "$OUT/$name" -o run --output-format csv -- "$@" \
        > "$OUT/$name.log" 2>&1 || fail "pmc pass $name" "$OUT/$name.log"
}

for task in "$@"; do
    IFS=: read -r -a A <<< "$task"
    case "${A[0]}" in
    tests)
        K=()
        [ -n "${A[1]}" ] && K=(-k "${A[1]}")
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${K[@]}" \
            > "$OUT/pytest_gpu.log" 2>&1 || fail tests "$OUT/pytest_gpu.log"
        tail -1 "$OUT/pytest_gpu.log" ;;
    smoke)
        timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 || fail smoke "$OUT/smoke.log"
        tail -1 "$OUT/smoke.log" ;;
    bench)
        timeout -k 10 600 python bench.py $BENCH_ARGS > "$OUT/bench.log" 2>&1 || fail bench "$OUT/bench.log"
        tail -1 "$OUT/bench.log" ;;
    rehearse)
        n=${A[1]:-2}
        RT_BENCH_DEVICE=0 timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node "$n" \
            --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus "$n" --steps 1 --warmup 0 $BENCH_ARGS \
            > "$OUT/rehearsal_n$n.log" 2>&1 || fail rehearse "$OUT/rehearsal_n$n.log"
        grep '^{"metric"' "$OUT/rehearsal_n$n.log" | tail -1 | cut -c1-400 ;;
    trace)
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- \
            python bench.py --no-cpu-baseline $BENCH_ARGS > "$OUT/trace.log" 2>&1 || fail trace "$OUT/trace.log"
        tail -1 "$OUT/trace.log" | cut -c1-300 ;;
    ktrace)
        script=${A[1]}
        KT=$((KT + 1))
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/ktrace_$KT" -o run --output-format csv -- \
            python "$script" "${A[@]:2}" > "$OUT/ktrace_$KT.log" 2>&1 || fail ktrace "$OUT/ktrace_$KT.log"
        tail -1 "$OUT/ktrace_$KT.log" | cut -c1-300
        find "$OUT/ktrace_$KT" -name "*kernel_stats.csv" -exec cut -d, -f1-5 {} \; | head -8 ;;
    benchpmc)
        # the bench command's own counters: HBM traffic (roofline.traffic; separate FETCH / WRITE passes)
        # and the VALU instruction mix + clock (roofline.compute), each pass a run of its own
        B=(python bench.py --steps 1 --warmup 0 --no-cpu-baseline $BENCH_ARGS)
        pmc_pass bench_fetch FETCH_SIZE GRBM_GUI_ACTIVE -- "${B[@]}"
        pmc_pass bench_write WRITE_SIZE -- "${B[@]}"
        pmc_pass bench_sq1 $SQ1 -- "${B[@]}"
        pmc_pass bench_sq2 $SQ2 -- "${B[@]}"
        pmc_pass bench_sq3 $SQ3 -- "${B[@]}"
        pmc_pass bench_w1 $SQW1 -- "${B[@]}"
        pmc_pass bench_w2 $SQW2 -- "${B[@]}"
        line=$(grep '^{"metric"' "$OUT/bench_fetch.log" | tail -1)
        key=$(echo "$line" | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['config']['workload'],d['config']['mode'])")
        # pmc_report.py reads the workload's sample / vertex counts and device time from a plain log
        echo "$line" | python -c "import json,sys;d=json.loads(sys.stdin.read());c=d['config'];s=c['width']*c['height']*c['traced_spp'];print(f\"bench: samples {s}, vertices {c['vertices']}, {d['roofline']['kernel_ms']} ms device\")" > "$OUT/bench_plain.log"
        python tools/pmc_traffic.py "$OUT/bench_fetch/run_counter_collection.csv" "$OUT/bench_write/run_counter_collection.csv" \
            "$key" --out "$OUT/pmc_traffic.json" || fail benchpmc
        python tools/pmc_report.py "$OUT" bench k_megakernel --out "$OUT/pmc_bench.json" --valu-key "$key" \
            --valu-out "$OUT/pmc_valu.json" > "$OUT/pmc_report.log" 2>&1 || fail "benchpmc report" "$OUT/pmc_report.log"
        echo "benchpmc $key ok" ;;
    configs)
        timeout -k 10 900 python -u tools/configs_bench.py > "$OUT/configs.log" 2>&1 || fail configs "$OUT/configs.log"
        cat "$OUT/configs.log" ;;
    pmc)
        scene=${A[1]}; w=${A[2]}; h=${A[3]}; spp=${A[4]}; extra=${A[5]}
        P=(python tools/prof_render.py "$scene" "$w" "$h" "$spp" mk $extra)
        key="${scene}_${w}x${h}x${spp}${extra:+_$extra}"
        timeout -k 10 120 "${P[@]}" > "$OUT/${key}_plain.log" 2>&1 || fail "plain $key" "$OUT/${key}_plain.log"
        cat "$OUT/${key}_plain.log"
        pmc_pass "${key}_fetch" FETCH_SIZE GRBM_GUI_ACTIVE -- "${P[@]}"
        pmc_pass "${key}_write" WRITE_SIZE -- "${P[@]}"
        pmc_pass "${key}_tcc" TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE -- "${P[@]}"
        pmc_pass "${key}_sq1" $SQ1 -- "${P[@]}"
        pmc_pass "${key}_sq2" $SQ2 -- "${P[@]}"
        pmc_pass "${key}_sq3" $SQ3 -- "${P[@]}"
        echo "pmc $key ok" ;;
    avail)
        # the counters rocprofv3 can collect on this device
        timeout -k 10 120 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1 || fail avail "$OUT/avail.txt"
        grep -c . "$OUT/avail.txt" ;;
    pmcw)
        # the wait breakdown of one megakernel render (two SQ passes, tools/pmc_report.py --waits)
        scene=${A[1]}; w=${A[2]}; h=${A[3]}; spp=${A[4]}; extra=${A[5]}
        P=(python tools/prof_render.py "$scene" "$w" "$h" "$spp" mk $extra)
        key="${scene}_${w}x${h}x${spp}${extra:+_$extra}"
        timeout -k 10 120 "${P[@]}" > "$OUT/${key}_plain.log" 2>&1 || fail "plain $key" "$OUT/${key}_plain.log"
        pmc_pass "${key}_w1" $SQW1 -- "${P[@]}"
        pmc_pass "${key}_w2" $SQW2 -- "${P[@]}"
        echo "pmcw $key ok" ;;
    dbgbuild)
        # diagnostic library (RT_DEBUG_COUNTERS + RT_DEBUG_TIMERS) at raytracer-server_amd/lib/variants/dbg.so
        make -s -j16 -C raytracer-server_amd BUILD=build_dbg LIB=lib/variants/dbg.so \
            EXTRA="-DRT_DEBUG_COUNTERS=1 -DRT_DEBUG_TIMERS=1 -DRT_AB_KNOBS=1" > "$OUT/dbgbuild.log" 2>&1 || fail dbgbuild "$OUT/dbgbuild.log"
        echo "dbg build ok" ;;
    env)
        # env:VAR=VAL[,VAR=VAL...] applies to the tasks after it (A/B runs of the RT_* switches)
        IFS=, read -r -a KV <<< "${task#env:}"
        for kv in "${KV[@]}"; do export "$kv"; echo "env $kv"; done ;;
    py)
        script=${A[1]}
        LOG="$OUT/$(basename "$script" .py).log"
        echo "== $task $(env | grep -E '^RT_' | tr '\n' ' ')" >> "$LOG"
        timeout -k 10 900 python -u "$script" "${A[@]:2}" > "$OUT/py_last.log" 2>&1 || { cat "$OUT/py_last.log" >> "$LOG"; fail "$script" "$OUT/py_last.log"; }
        cat "$OUT/py_last.log" >> "$LOG"
        tail -40 "$OUT/py_last.log" ;;
    *)
        fail "unknown task $task" ;;
    esac
done
echo "gpu_task: all done ($*)"

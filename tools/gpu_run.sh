#!/bin/bash
# The one lease runner (replaces the round-1/2 one-off gpu_*.sh scripts).
# Runs on the GPU box through gpurun, from the repo root:
#   gpurun --timeout 900 -- bash tools/gpu_run.sh <step> [<step> ...]
# Each step runs under its own time limit; the first failing step ends the
# call (no GPU step runs after a failure, a fault or a time limit).
# Steps (arguments separated by ':'):
#   tests:<tag>[:<pytest selector>]  GPU tests -> gpurun_out/t_<tag>.log ("@" stands for "::",
#                                    "~" separates node ids)
#   bench:<tag>[:<bench.py args, ',' for ' '>]  -> gpurun_out/bench_<tag>.json/.err
#   profile:<tag>:<config>:<steps>   kernel trace + FETCH/WRITE/SQ PMC passes of the
#                                    timed bench steps -> gpurun_out/prof_<tag>/
#   pmclds:<tag>:<config>:<steps>    the LDS counter pass (SQ_INSTS_LDS, bank conflicts, ...)
#                                    -> gpurun_out/prof_<tag>/lds/
#   py:<tag>:<script>[:<args, "~" for " ">]  a tools/ script -> gpurun_out/<tag>.log
#   pyenv:<tag>:<VAR=v~VAR2=v>:<script>[:<args>]  the same with environment variables
#   kstats:<tag>:<script>:<args>[:<counters>]  the script under rocprofv3 (kernel trace + stats,
#                                    or one --pmc pass) -> gpurun_out/ks_<tag>/
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out

run_tests() {  # tag selector ("@" for "::" and "~" for " ": the step itself is split at ':')
    local tag=$1 sel=${2:-tests}
    sel=${sel//@/::}
    sel=${sel//\~/ }
    echo "[gpu_run] tests $tag: $sel"
    timeout -k 10 900 python -u -m pytest $sel -m gpu -x -v --timeout 180 --timeout-method thread \
        > gpurun_out/t_$tag.log 2>&1 || { tail -40 gpurun_out/t_$tag.log; return 1; }
    tail -1 gpurun_out/t_$tag.log
}

run_bench() {  # tag args
    local tag=$1 args=${2//,/ }
    echo "[gpu_run] bench $tag: $args"
    timeout -k 10 600 python -u bench.py $args > gpurun_out/bench_$tag.json 2> gpurun_out/bench_$tag.err \
        || { tail -30 gpurun_out/bench_$tag.err; return 1; }
    cut -c1-600 gpurun_out/bench_$tag.json
}

run_profile() {  # tag config steps
    local tag=$1 cfg=${2:-3} steps=${3:-20}
    local out=gpurun_out/prof_$tag
    local B="bench.py --only-timed --no-cpu-baseline --no-extra --config $cfg --steps $steps --warmup 3"
    echo "[gpu_run] profile $tag: config $cfg, $steps steps"
    mkdir -p $out
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -- python3 $B \
        > $out/trace.log 2>&1 || { tail -20 $out/trace.log; return 1; }
    timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -- python3 $B \
        > $out/fetch.log 2>&1 || { tail -20 $out/fetch.log; return 1; }
    timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $out/write -- python3 $B \
        > $out/write.log 2>&1 || { tail -20 $out/write.log; return 1; }
    timeout -k 10 300 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_THREAD_CYCLES_VALU \
        SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE --output-format csv -d $out/sq -- python3 $B \
        > $out/sq.log 2>&1 || { tail -20 $out/sq.log; return 1; }
    echo "[gpu_run] profile $tag done"
}

run_pmclds() {  # tag config steps: the LDS/issue counter pass (its own step, so a counter
                # the box lacks ends only this step) -> gpurun_out/prof_<tag>/lds
    local tag=$1 cfg=${2:-3} steps=${3:-20}
    local out=gpurun_out/prof_$tag
    local B="bench.py --only-timed --no-cpu-baseline --no-extra --config $cfg --steps $steps --warmup 3"
    echo "[gpu_run] pmclds $tag: config $cfg, $steps steps"
    mkdir -p $out
    timeout -k 10 -s KILL 300 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS \
        SQ_BUSY_CYCLES SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d $out/lds -- python3 $B \
        > $out/lds.log 2>&1 || { tail -20 $out/lds.log; return 1; }
    echo "[gpu_run] pmclds $tag done"
}

run_kstats() {  # tag script args [pmc counters, "~" for " "]: a tools/ script under rocprofv3
                # (kernel trace + stats; with counters, one --pmc pass instead) -> gpurun_out/ks_<tag>/
    local tag=$1 script=$2 args=${3//\~/ } pmc=${4//\~/ }
    local out=gpurun_out/ks_$tag
    mkdir -p $out
    if [ -z "$pmc" ]; then
        echo "[gpu_run] kstats $tag: $script $args"
        timeout -k 10 -s KILL 600 rocprofv3 --kernel-trace --stats --output-format csv -d $out -- python3 $script $args \
            > $out/run.log 2>&1 || { tail -20 $out/run.log; return 1; }
    else
        echo "[gpu_run] kstats $tag (pmc $pmc): $script $args"
        timeout -k 10 -s KILL 600 rocprofv3 --pmc $pmc --output-format csv -d $out -- python3 $script $args \
            > $out/run.log 2>&1 || { tail -20 $out/run.log; return 1; }
    fi
    tail -3 $out/run.log
}

run_py() {  # tag script args
    local tag=$1 script=$2 args=${3//\~/ }
    echo "[gpu_run] py $tag: $script $args"
    timeout -k 10 900 python -u $script $args > gpurun_out/$tag.log 2>&1 || { tail -40 gpurun_out/$tag.log; return 1; }
    tail -5 gpurun_out/$tag.log
}

run_pyenv() {  # tag env-assignments ("~" between) script args: a tools/ script with environment variables
    local tag=$1 envs=${2//\~/ } script=$3 args=${4//\~/ }
    echo "[gpu_run] pyenv $tag: $envs $script $args"
    env $envs timeout -k 10 900 python -u $script $args > gpurun_out/$tag.log 2>&1 || { tail -40 gpurun_out/$tag.log; return 1; }
    tail -5 gpurun_out/$tag.log
}

for step in "$@"; do
    IFS=':' read -r kind a b c d <<< "$step"
    case $kind in
        tests) run_tests "$a" "$b" || exit 1 ;;
        bench) run_bench "$a" "$b" || exit 1 ;;
        profile) run_profile "$a" "$b" "$c" || exit 1 ;;
        pmclds) run_pmclds "$a" "$b" "$c" || exit 1 ;;
        py) run_py "$a" "$b" "$c" || exit 1 ;;
        pyenv) run_pyenv "$a" "$b" "$c" "$d" || exit 1 ;;
        kstats) run_kstats "$a" "$b" "$c" "$d" || exit 1 ;;
        *) echo "unknown step $step"; exit 2 ;;
    esac
done

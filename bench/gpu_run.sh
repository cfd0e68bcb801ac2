#!/bin/bash
# One parametrised GPU-session script (it replaces the per-round bench/gpu_r0*.sh one-offs). Every step runs under
# its own time limit and writes under gpurun_out/; the first failing step ends the session (set -e).
#   bash bench/gpu_run.sh <tag> <step> [<step> ...]
# steps:
#   tests                  the whole GPU suite (pytest -m gpu)
#   tests:<expr>           the GPU tests matching a pytest -k expression
#   smoke                  __graft_entry__.smoke()
#   bench[:<args>]         python bench.py <args>            -> gpurun_out/bench_<tag>_<i>.json
#   config:<args>          python bench/bench_configs.py <args> -> gpurun_out/config_<tag>_<i>.json
#   rocprof[:<args>]       rocprofv3 --kernel-trace --stats of python3 bench.py <args> -> gpurun_out/prof_<tag>_<i>/
#   rocprofcfg:<args>      the same of python3 bench/bench_configs.py <args>        -> gpurun_out/prof_<tag>_<i>/
#   pmc:<counters>[@<args>] one rocprofv3 --pmc pass of bench.py <args> -> gpurun_out/pmc_<tag>_<i>/
#   pmccfg:<counters>@<args> one rocprofv3 --pmc pass of bench/bench_configs.py <args> -> gpurun_out/pmc_<tag>_<i>/
#   py:<script args>       python <script args>              -> gpurun_out/py_<tag>_<i>.log
#   rocprofpy:<script args> rocprofv3 --kernel-trace --stats of python3 <script args> -> gpurun_out/prof_<tag>_<i>/
#   env:<NAME>=<value>     export a variable for the steps after it (env:NAME= clears it)
#   sh:<script args>       bash <script args> (bench/pmc.sh, bench/bisect_sweep.sh: they time-limit their own steps)
set -euo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p "$O"
cd "$R"
export TMPDIR=/tmp
T=$1
shift
i=0
for step in "$@"; do
  i=$((i + 1))
  kind=${step%%:*}
  arg=""
  [[ "$step" == *:* ]] && arg=${step#*:}
  echo "[$T] step $i: $step ($(date +%T))"
  case "$kind" in
    tests)
      if [ -n "$arg" ]; then
        timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$arg" \
          > "$O/tests_${T}_$i.log" 2>&1
      else
        timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
          > "$O/tests_${T}_$i.log" 2>&1
      fi
      tail -3 "$O/tests_${T}_$i.log" ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke_${T}_$i.log" 2>&1 ;;
    bench)
      timeout -k 10 600 python bench.py $arg > "$O/bench_${T}_$i.json" 2> "$O/bench_${T}_$i.err"
      cut -c1-400 "$O/bench_${T}_$i.json" ;;
    config)
      timeout -k 10 600 python bench/bench_configs.py $arg > "$O/config_${T}_$i.json" 2> "$O/config_${T}_$i.err"
      cut -c1-400 "$O/config_${T}_$i.json" ;;
    rocprof)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_${T}_$i" -o run -- python3 bench.py $arg \
        > "$O/prof_${T}_$i.json" 2> "$O/prof_${T}_$i.err" ;;
    rocprofcfg)
      timeout -k 10 900 rocprofv3 --kernel-trace --stats -d "$O/prof_${T}_$i" -o run -- python3 bench/bench_configs.py $arg \
        > "$O/prof_${T}_$i.json" 2> "$O/prof_${T}_$i.err" ;;
    pmc)
      ctr=${arg%%@*}
      bargs=""
      [[ "$arg" == *@* ]] && bargs=${arg#*@}
      timeout -s KILL 300 rocprofv3 --pmc $ctr -d "$O/pmc_${T}_$i" -o run -- python3 bench.py $bargs \
        > "$O/pmc_${T}_$i.json" 2> "$O/pmc_${T}_$i.err" ;;
    pmccfg)
      ctr=${arg%%@*}
      cargs=""
      [[ "$arg" == *@* ]] && cargs=${arg#*@}
      timeout -s KILL 300 rocprofv3 --pmc $ctr -d "$O/pmc_${T}_$i" -o run -- python3 bench/bench_configs.py $cargs \
        > "$O/pmc_${T}_$i.json" 2> "$O/pmc_${T}_$i.err" ;;
    py)
      timeout -k 10 600 python $arg > "$O/py_${T}_$i.log" 2>&1
      tail -5 "$O/py_${T}_$i.log" ;;
    rocprofpy)
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$O/prof_${T}_$i" -o run -- python3 $arg \
        > "$O/prof_${T}_$i.log" 2>&1
      tail -3 "$O/prof_${T}_$i.log" ;;
    env)
      export "$arg" ;;
    sh)
      bash $arg ;;
    *)
      echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[$T] done ($(date +%T))"

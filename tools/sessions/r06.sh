#!/bin/bash
# Round-6 GPU sessions (run through gpurun from the repo root): tools/sessions/r06.sh <tag> <step>...
# steps: tests:<pytest -k expr or file> | bench | benchdef | prof | pmc | kprobe:<args>
# Every GPU step has its own time limit; the chain stops at the first failure.
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
step() { echo "[$(date +%T)] $*"; }
n=0
for s in "$@"; do
    n=$((n + 1))
    case "$s" in
    tests:*)
        sel=${s#tests:}
        step "pytest $sel"
        timeout -k 10 900 python -u -m pytest $sel -m gpu -x -q --timeout 300 --timeout-method thread > "$OUT/pytest_$n.log" 2>&1 || { tail -40 "$OUT/pytest_$n.log"; exit 1; }
        tail -3 "$OUT/pytest_$n.log" ;;
    bench)
        step "bench (driver flags)"
        timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench_$n.json" 2> "$OUT/bench_$n.err" || { tail -20 "$OUT/bench_$n.err"; exit 1; }
        cat "$OUT/bench_$n.json" ;;
    benchdef)
        step "bench (defaults)"
        timeout -k 10 600 python bench.py > "$OUT/benchdef_$n.json" 2> "$OUT/benchdef_$n.err" || { tail -20 "$OUT/benchdef_$n.err"; exit 1; }
        cat "$OUT/benchdef_$n.json" ;;
    prof)
        step "rocprof kernel trace of the bench (driver flags, no cpu leg)"
        timeout -k 10 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof_$n" -o run --output-format csv -- \
            python bench.py --steps 20 --warmup 5 --cpu-sweeps 0 > "$OUT/bench_prof_$n.json" 2> "$OUT/bench_prof_$n.err" || { tail -20 "$OUT/bench_prof_$n.err"; exit 1; } ;;
    py:*)
        cmd=${s#py:}
        step "python $cmd"
        timeout -k 10 600 python -u $cmd > "$OUT/py_$n.log" 2>&1 || { tail -30 "$OUT/py_$n.log"; exit 1; }
        tail -40 "$OUT/py_$n.log" ;;
    *) echo "unknown step $s"; exit 2 ;;
    esac
done
step done

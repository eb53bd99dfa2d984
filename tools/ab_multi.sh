#!/bin/bash
# bench.py V-cycle / pair under several values of one environment variable, interleaved (through gpurun):
#   tools/ab_multi.sh <tag> <VAR> "<v1> <v2> ..." [reps] [bench.py args...]
set -o pipefail
TAG=$1; VAR=$2; VALS=$3; REPS=${4:-2}; shift 4
O=gpurun_out/$TAG; mkdir -p $O
for rep in $(seq 1 $REPS); do for val in $VALS; do
  env "$VAR=$val" timeout -k 10 300 python bench.py --steps 20 --vcycles 100 --cpu-sweeps 0 --newton-iters 0 "$@" > $O/b_${val}_$rep.json 2>$O/b_${val}_$rep.err || { tail -20 $O/b_${val}_$rep.err; exit 1; }
  echo "$VAR=$val $(python tools/bench_brief.py $O/b_${val}_$rep.json)"
done; done

#!/bin/bash
# Round-2 GPU session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Each step under its own time limit; stops at the first step that ends in
# anything but success / test failure (rc 0 or 1).
cd "$GRAFT_REPO_ROOT" || exit 1
OUT="$GRAFT_REPO_ROOT/gpurun_out"
mkdir -p "$OUT"
export TMPDIR=/tmp
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "== $name: $*" >> "$OUT/steps.log"
  timeout -k 10 "$to" "$@" > "$OUT/$name.out" 2> "$OUT/$name.err"
  local rc=$?
  echo "== $name rc=$rc" >> "$OUT/steps.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name rc=$rc" >> "$OUT/steps.log"; exit $rc; fi
  return 0
}
MODE=${1:-all}
if [[ "$MODE" == *info* ]] || [ "$MODE" = all ]; then
  nproc > "$OUT/nproc.txt"; lscpu > "$OUT/lscpu.txt" 2>&1
  echo "OMP_NUM_THREADS=$OMP_NUM_THREADS" >> "$OUT/nproc.txt"
fi
if [[ "$MODE" == *tests* ]] || [ "$MODE" = all ]; then
  step tests 600 python -u -m pytest tests -m gpu -x -v -rf --timeout 400 --timeout-method thread ${TESTS_K:+-k "$TESTS_K"}
  step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [[ "$MODE" == *bench* ]] || [ "$MODE" = all ]; then
  step bench 700 python bench.py ${BENCH_ARGS}
fi
if [[ "$MODE" == *prof* ]]; then
  step prof_bench 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_bench" -o bench -- python3 "$GRAFT_REPO_ROOT/bench.py" --no-e2e
fi
if [[ "$MODE" == *pipetrace1* ]]; then
  # one launching thread: the traced pipe path (the multi-threaded legs
  # crash the tracer, profiles/README.md)
  step prof_pipe1 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_pipe1" -o pipe -- python3 "$GRAFT_REPO_ROOT/bench.py" --only pipe --pipe-threads 1
elif [[ "$MODE" == *pipetrace* ]]; then
  step prof_pipe 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/prof_pipe" -o pipe -- python3 "$GRAFT_REPO_ROOT/bench.py" --only pipe
fi
echo done >> "$OUT/steps.log"

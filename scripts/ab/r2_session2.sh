# r2 measurement session: GPU suite, smoke, headline bench, 64-client bench + round
# time series, first-write probe, rocprof kernel trace of the headline bench
set -u
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$ROOT"
export HSA_ENABLE_IPC_MODE_LEGACY=0
OUT=gpurun_out/s2
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 1; }
tail -1 $OUT/pytest_gpu.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --steps 50 --warmup 5 --out $OUT/bench.json > $OUT/bench.log 2>&1 || exit $?
timeout -k 10 300 python scripts/bench_kernels.py > $OUT/bench_kernels.log 2>&1 || exit $?
FEDMX_WRITER_STATS=1 timeout -k 10 180 python bench.py --clients 64 --data-kind kitsune --non-iid --steps 50 --warmup 5 --out $OUT/kitsune64.json > $OUT/kitsune64.log 2> $OUT/kitsune64.err || exit $?
timeout -k 10 200 python scripts/round_time_series.py --non-iid --rounds 70 > $OUT/k64_series.json 2> $OUT/k64_series.err || exit $?
timeout -k 10 100 python scripts/first_write_probe.py > $OUT/first_write.json 2>&1 || exit $?
timeout -k 10 180 python bench.py --epochs 100 --lr 1e-5 --shrink-lambda 10 --steps 20 --warmup 3 --out $OUT/paper.json > $OUT/paper.log 2>&1 || exit $?
NRANKS=4 bash scripts/multirank_rehearsal.sh > $OUT/rehearsal4.txt 2>&1 || { cat $OUT/rehearsal4.txt; exit 1; }
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$ROOT/$OUT/prof" -o run -- python3 "$ROOT/bench.py" --steps 5 --warmup 2 > "$ROOT/$OUT/rocprof.log" 2>&1

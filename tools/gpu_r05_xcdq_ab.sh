# int8 column quantiser (bn_dz_quant_cols_t_k) with the XCD remap (in-tree library) against HEAD
# (abv/base): parity tests of the s20 / pixel paths, then default-bench runs with the kernel
# timers, alternating, 3 rounds.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_s20.py tests/test_gpu_pixels.py > gpurun_out/r05_xcdq_tests.log 2>&1 \
  || { echo "TESTS FAIL"; tail -30 gpurun_out/r05_xcdq_tests.log; exit 1; }
tail -2 gpurun_out/r05_xcdq_tests.log
for r in 1 2 3; do
  for v in A B; do
    case $v in A) export BNN_LIB=$GRAFT_REPO_ROOT/abv/base/libbnn.so;; G) export BNN_LIB=$GRAFT_REPO_ROOT/abv/guard/libbnn.so;; B) unset BNN_LIB;; esac
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_xcdq_$v$r.log 2>&1 || { echo "RUN $v$r FAIL"; tail -5 gpurun_out/r05_xcdq_$v$r.log; exit 1; }
    tail -1 gpurun_out/r05_xcdq_$v$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$v$r', d['ms_per_step'], ' | '.join(f'{n[:40]}={v[\"avg_us\"]:.0f}' for n,v in k.items() if 'i8cols' in n or 'q6' in n))"
  done
done
# FETCH_SIZE of the quantiser on the in-tree library (one pass)
cd /tmp && export TMPDIR=/tmp && unset BNN_LIB && mkdir -p $GRAFT_REPO_ROOT/gpurun_out/r05_xcdq_pmc
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/gpurun_out/r05_xcdq_pmc/fetch -o fetch --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 1 --warmup 1 --no-cpu-baseline --no-gpu-torch --no-kernel-timing --no-dropin > $GRAFT_REPO_ROOT/gpurun_out/r05_xcdq_pmc/fetch.log 2>&1 || { echo "PMC FAIL"; tail -5 $GRAFT_REPO_ROOT/gpurun_out/r05_xcdq_pmc/fetch.log; exit 1; }
python3 $GRAFT_REPO_ROOT/tools/pmc_table.py $GRAFT_REPO_ROOT/gpurun_out/r05_xcdq_pmc dz_quant

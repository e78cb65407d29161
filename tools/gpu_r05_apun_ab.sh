# Two streaming-pass A/Bs in one run, default-bench kernel timers, alternating, 3 rounds:
#  - bn_apply_pack_fp4_k phase-1 unroll (rows whose loads are in flight together): 4 (abv/rb8) against
#    8 (abv/ap8) and 16 (abv/ap16);
#  - the forward statistics pass on z16 in 16-row load batches (in-tree) against 8 (abv/rb8).
# Keep-bit / statistics parity tests on the in-tree library first.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_keep_bits.py tests/test_gpu_z16.py tests/test_gpu_fused.py > gpurun_out/r05_apun_tests.log 2>&1 \
  || { echo "TESTS FAIL"; tail -30 gpurun_out/r05_apun_tests.log; exit 1; }
tail -2 gpurun_out/r05_apun_tests.log
for r in 1 2 3; do
  for v in rb8 ap8 ap16 new; do
    if [ $v = new ]; then unset BNN_LIB; else export BNN_LIB=$GRAFT_REPO_ROOT/abv/$v/libbnn.so; fi
    timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_apun_$v$r.log 2>&1 || { echo "RUN $v$r FAIL"; tail -5 gpurun_out/r05_apun_$v$r.log; exit 1; }
    tail -1 gpurun_out/r05_apun_$v$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('$v$r', d['ms_per_step'], ' | '.join(f'{n[:40]}={v[\"avg_us\"]:.0f}' for n,v in k.items() if 'apply' in n or 'fwd' in n or 'stats' in n))"
  done
done

# Parity of the q6 / head / keep-bit / z16 paths and the config-5 step after the q6 prefetch change.
set -o pipefail
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 1000 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_gpu_keep_bits.py tests/test_gpu_z16.py tests/test_gpu_q6_handoff.py tests/test_gpu_head.py tests/test_gpu_fp6.py tests/test_gpu_wide_step.py tests/test_gpu_fused.py > gpurun_out/r05_q6tests.log 2>&1 || { echo TESTS FAIL; tail -30 gpurun_out/r05_q6tests.log; exit 1; }
tail -2 gpurun_out/r05_q6tests.log
# the u8-pixel statistics GEMM's tile: 128 x 128 (BNN_PIX_TILE=1) against the default 256 x 256,
# alternating default-bench runs with the bench kernel timers
for r in 1 2; do
  for v in 1 0; do
    BNN_PIX_TILE=$v timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-gpu-torch --no-dropin > gpurun_out/r05_pixtile_$v$r.log 2>&1 || { echo "RUN $v$r FAIL"; tail -5 gpurun_out/r05_pixtile_$v$r.log; exit 1; }
    tail -1 gpurun_out/r05_pixtile_$v$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); k=d['kernels']; print('tile$v r$r', d['ms_per_step'], ' | '.join(f'{n[:44]}={v[\"avg_us\"]:.0f}' for n,v in k.items() if 'pixel' in n or 'i8' in n or 'fc1' in n or 'bn_fwd' in n))"
  done
done

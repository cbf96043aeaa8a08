cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out && timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q -k "gemm_tile" -p no:cacheprovider > gpurun_out/pytest_gemm_tile.log 2>&1 && timeout -k 10 300 python -u scripts/bench_gemm_stream.py 256 128 > gpurun_out/bench_gemm_stream.log 2>&1
rc=$?; tail -n 5 gpurun_out/pytest_gemm_tile.log; cat gpurun_out/bench_gemm_stream.log; exit $rc

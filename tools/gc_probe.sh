cd $GRAFT_REPO_ROOT
timeout -k 10 300 python3 -c "import gc, sys; gc.disable(); import pytest; sys.exit(pytest.main(['tests', '-m', 'gpu', '-x', '-q', '-p', 'no:timeout', '-k', 'test_gpu_model']))" > gpurun_out/gc0.log 2>&1; echo "gc disabled rc=$?"; grep -E "passed|failed|Fatal" gpurun_out/gc0.log | head -3
timeout -k 10 300 python3 -c "import gc, sys; import pytest; sys.exit(pytest.main(['tests', '-m', 'gpu', '-x', '-q', '-p', 'no:timeout', '-k', 'test_gpu_model']))" > gpurun_out/gc1.log 2>&1; echo "gc enabled rc=$?"; grep -E "passed|failed|Fatal" gpurun_out/gc1.log | head -3
exit 0

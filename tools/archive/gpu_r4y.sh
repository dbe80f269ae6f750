# Round-4 GPU pass y: the host code under ASan/UBSan (big epochs drive every parallel commit
# phase) and ThreadSanitizer (tests/native/tsan_engine), then the GPU suite ('+' edges placed
# after their parent's slot).
set -o pipefail
T=${1:-y}
mkdir -p gpurun_out
timeout -k 10 600 ./tests/native/asan_driver > gpurun_out/asan_$T.log 2>&1
rc=$?; tail -3 gpurun_out/asan_$T.log; [ $rc -eq 0 ] || exit $rc
TSAN_OPTIONS="halt_on_error=0 report_signal_unsafe=0 second_deadlock_stack=1 log_path=gpurun_out/tsan_$T" \
  timeout -k 10 600 ./tests/native/tsan_engine > gpurun_out/tsan_$T.out 2>&1
rc=$?; tail -3 gpurun_out/tsan_$T.out; ls gpurun_out/ | grep "tsan_$T" | head -3; [ $rc -eq 0 ] || [ $rc -eq 66 ] || exit $rc
timeout -k 10 900 python -u -m pytest -v --timeout 420 --timeout-method thread tests -m gpu -x > gpurun_out/pytest_gpu_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_gpu_$T.log; grep -E "FAILED|Error" gpurun_out/pytest_gpu_$T.log | head -20; exit $rc

# Round-4 GPU pass y: the host code under ASan/UBSan (big epochs now drive every parallel
# commit phase) and under ThreadSanitizer (tests/native/tsan_engine, built in this container).
set -o pipefail
T=${1:-y}
mkdir -p gpurun_out
timeout -k 10 600 ./tests/native/asan_driver > gpurun_out/asan_$T.log 2>&1
rc=$?; tail -5 gpurun_out/asan_$T.log; [ $rc -eq 0 ] || exit $rc
TSAN_OPTIONS="halt_on_error=0 report_signal_unsafe=0 second_deadlock_stack=1 log_path=gpurun_out/tsan_$T" \
  timeout -k 10 900 ./tests/native/tsan_engine > gpurun_out/tsan_$T.out 2>&1
rc=$?; tail -5 gpurun_out/tsan_$T.out; ls gpurun_out/ | grep tsan_$T | head; exit $rc

# Round-4 GPU pass v: image checks at parallel-phase sizes and in the full-size E churn test.
set -o pipefail
T=${1:-v}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -v --timeout 600 --timeout-method thread tests/test_gpu_image.py tests/test_gpu_fullsize.py -k "image or config_e" -x > gpurun_out/pytest_image_$T.log 2>&1
rc=$?; tail -n 3 gpurun_out/pytest_image_$T.log; grep -E "FAILED|Error|assert" gpurun_out/pytest_image_$T.log | head -10; exit $rc

# round 6: the checked dense pull (tests, then A/B against the gather-only pull), then the whole suite
set -o pipefail
O=gpurun_out/r06n
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_slab.py -m gpu -x -v --timeout 240 --timeout-method thread -k "checked_dense_pull or two_streams or adaptive_switch_and_errors or fine_stage or set_push" > $O/pytest_new.log 2>&1 || exit 1
TAG=r06n_pull STAGES=abn PATTERNS=pull ROUNDS=3 LIBS="old=tools/ablibs/libglint_gpu_prevpull.so cur=glint_amd/lib/libglint_gpu.so sb1=tools/ablibs/libglint_gpu_sb1.so sb4=tools/ablibs/libglint_gpu_sb4.so" bash tools/gpu_run.sh || exit 1
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > $O/suite.log 2>&1 || exit 1

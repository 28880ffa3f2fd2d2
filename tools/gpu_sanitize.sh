# Host-side ASan/UBSan stress test of libtkv_crc32's host paths (tests/cpp/test_host_paths.cpp,
# built on the box by `make -C tinykvpp_amd/csrc sanitize`; tests/cpp/build does not travel).
# Device code is not instrumented.
set -e
R=$GRAFT_REPO_ROOT
cd $R
mkdir -p gpurun_out/san
make -s -C tinykvpp_amd/csrc sanitize -j8 > gpurun_out/san/build.log 2>&1
export ASAN_OPTIONS=detect_leaks=0:protect_shadow_gap=0:halt_on_error=1
export UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
timeout -k 10 300 tests/cpp/build/test_host_paths_san > gpurun_out/san/sanitize.log 2>&1

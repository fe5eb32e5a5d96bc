// daxpy_nvtx — daxpy with roctx ranges (copyInput, cublasDaxpy, copyOutput)
// and a roctx profiler capture window, the MI355X equivalent of the
// reference's NVTX + cudaProfilerStart/Stop (daxpy_nvtx.cu:65-105).
// Profile with: rocprofv3 --marker-trace --kernel-trace -- build/bin/daxpy_nvtx
#include "daxpy_common.hpp"

int main(int argc, char** argv) { return gmt::apps::daxpy_main(argc, argv, true); }

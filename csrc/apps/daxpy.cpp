// daxpy — single-GPU DAXPY probe (reference daxpy.cu:35-94); body in daxpy_common.hpp.
#include "daxpy_common.hpp"

int main(int argc, char** argv) { return gmt::apps::daxpy_main(argc, argv, false); }

// Test harness: the product's fixed-point formatter (taxi2_amd/csrc/format_kernels.hpp) compiled
// for the host, checked against Python's '%.Nf' by tests/test_writers_native.py.
#include "../../taxi2_amd/csrc/format_kernels.hpp"

extern "C" int fmt_host(double x, int n, char* dst) { return taxi2::fmt_fixed(x, n, dst); }

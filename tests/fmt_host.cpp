// Host build of csrc/fmt_float.h for the CPU tests (test infrastructure only): the formatter is
// device code in the library; here `__device__` is defined away so the same source runs on the
// host against Python's shortest-repr digits (tests/test_encode.py).
#define __device__
#include "fmt_float.h"

extern "C" int fmt_f64_c(double v, char *out) { return qeh::fmt_f64(out, v); }
extern "C" int fmt_f32_c(float v, char *out) { return qeh::fmt_f32(out, v); }
extern "C" int fmt_i64_c(long long v, char *out) { return qeh::fmt_i64(out, v); }

// fcx_match_k4.hip — k_match with the bucket search over 4-byte keys (k_match_k4 / launch_match_k4):
// the dense-key translation unit of fcx_match.hip (see FCX_KEY4 there).  A unit of its own, so the
// 3-byte kernel's source and code stay as they are.
#define FCX_KEY4 1
#include "fcx_match.hip"

// fcx_match_k4.hip — k_match with the bucket search over 4-byte keys (k_match_k4 / launch_match_k4):
// the dense-key translation unit of fcx_match.hip (see FCX_KEY4 there).  Small-alphabet tiles always
// reach the bucket search, so the unit also drops the repeat filter and the run count
// (FCX_NOFILTER; dna k_match 25.0 -> 24.4 ms per GiB).  A unit of its own, so the general kernel's
// source and code stay as they are.
#define FCX_KEY4 1
#define FCX_NOFILTER 1
#define FCX_UNIT_ILP 2   // two interleaved bucket walks per lane: dna k_match 24.6 -> 24.0 ms per GiB
#include "fcx_match.hip"

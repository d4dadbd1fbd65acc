// fcx_match_runs.hip — k_match with the run-mode walk inlined (k_match_runs / launch_match_runs): the
// long-match (runs, zeros) translation unit of fcx_match.hip (see FCX_RUNS there).  A unit of its
// own, so the general kernel's source and code stay as they are.
#define FCX_RUNS 1
#include "fcx_match.hip"

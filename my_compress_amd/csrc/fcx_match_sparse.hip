// fcx_match_sparse.hip — k_match without the bucket search (k_match_sparse / launch_match_sparse): the
// few-match (random data) translation unit of fcx_match.hip (see FCX_SPARSE there).  A unit of its
// own, so the general kernel's source and code stay as they are.
#define FCX_SPARSE 1
#include "fcx_match.hip"

// fcx_match_nf.hip — k_match without the repeat sample, filter and sparse search (k_match_nf /
// launch_match_nf): the match-dense (text) translation unit of fcx_match.hip (see FCX_NOFILTER there).
// A unit of its own, so the general kernel's source and code stay as they are.
#define FCX_NOFILTER 1
#define FCX_UNIT_ILP 2   // two interleaved walks per lane: text k_match 9.95 -> 9.67 ms per GiB (4: 0 spills,
                         // but the wider walk pays on text's short buckets)
#include "fcx_match.hip"

// fcx_match_runs.hip — k_match with the run-mode walk inlined (k_match_runs / launch_match_runs): the
// long-match (runs, zeros) translation unit of fcx_match.hip (see FCX_RUNS there).  Its shards' tiles
// take the run mode or the sparse search, so the unit also drops the bucket search (FCX_NOBUCKET: a
// tile that takes neither takes the whole-tile run-table mode; runs k_match 8.97 -> 8.83 ms per GiB,
// zeros 1.92 -> 1.82) and the repeat sample (a tile that is not run mode always runs the filter;
// zeros 1.83 -> 1.63, runs 8.82 -> 8.76).  A unit of its own, so the general kernel's source and
// code stay as they are.
#define FCX_RUNS 1
#define FCX_NOBUCKET 1
#include "fcx_match.hip"

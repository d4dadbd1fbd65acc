# A/B of library variants: devbench stage times per leg for lib/libfcx.so (A) and each
# lib/libfcx_<V>.so in $VARS (FCX_LIB), e.g. VARS="x y" KINDS="rand text c3" bash tools/gpu_ab.sh
set -u
# timing-exit builds (tools/phase_libs.sh: libfcx_x<N>.so, FCX_MATCH_EXIT) leave the scratch the later
# kernels read unwritten: they are for the kernel-alone timing (tools/gpu_match_phases.sh), never the
# whole pipeline run here
for v in ${VARS:-b}; do
  case $v in x*) echo "gpu_ab.sh: refusing timing-exit variant libfcx_$v.so (use tools/gpu_match_phases.sh)" >&2; exit 2;; esac
done
for leg in ${KINDS:-rand text dna runs}; do
  case $leg in
    text) a="--kind text --seed 3 --mib 1024 --check hl_text_1GiB";;
    rand) a="--kind rand --seed 4 --mib 1024 --check hl_rand_1GiB";;
    runs) a="--kind runs --seed 5 --mib 1024 --check cfg5b_runs_1GiB";;
    zeros) a="--kind zeros --seed 0 --mib 1024 --check cfg5a_zeros_1GiB";;
    dna) a="--kind dna --seed 6 --mib 1024";;
    c3) a="--kind text --seed 3 --mib 1024 --block 262144 --check cfg3_text_1GiB";;
    c2) a="--kind rand --seed 2 --mib 64 --block 65536 --check cfg2_rand_64MiB";;
  esac
  timeout -k 10 200 python tools/devbench.py $a > gpurun_out/ab_A_$leg.log 2>&1 || exit 1
  for v in ${VARS:-b}; do
    FCX_LIB=$PWD/my_compress_amd/lib/libfcx_$v.so timeout -k 10 200 python tools/devbench.py $a > gpurun_out/ab_${v}_$leg.log 2>&1 || exit 1
  done
done

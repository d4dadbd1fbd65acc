# summary of tools/gpu_ab.sh logs: VARS="..." KINDS="..." bash tools/gpu_ab_summary.sh
for k in ${KINDS:-rand text dna runs}; do for v in A ${VARS:-b}; do printf "%-5s %-6s " $k $v; grep -o "groups 0:.*GB/s\|match [0-9.]*\|emit [0-9.]*\|digest [A-Z]*" gpurun_out/ab_${v}_$k.log 2>/dev/null | tr '\n' ' '; echo; done; done

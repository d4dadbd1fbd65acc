# summary of tools/gpu_check.sh logs
tail -1 gpurun_out/gs_parity.log
for f in rand c2 text c3 runs zeros dna; do printf "%-6s " $f; grep -o "groups 0:.*GB/s\|digest [A-Z]*\|match [0-9.]*\|stitch [0-9.]*\|emit [0-9.]*\|tree [0-9.]*\|encode [0-9.]*" gpurun_out/gs_$f.log | tr '\n' ' '; echo; done

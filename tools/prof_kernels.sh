# rocprofv3 kernel stats of tools/devbench.py for the kinds in $KINDS (kind:seed), one run each
set -u
R=$PWD
export TMPDIR=/tmp
for leg in ${KINDS:-rand:4}; do
  IFS=: read kind seed <<< "$leg"
  (cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/pk_$kind -o run --output-format csv -- python3 $R/tools/devbench.py --kind $kind --seed $seed --mib 1024 > $R/gpurun_out/pk_$kind.log 2>&1) || exit 1
done

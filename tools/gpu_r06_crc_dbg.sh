set -o pipefail
cd $GRAFT_REPO_ROOT; export TMPDIR=/tmp
for dbg in 0 1 2 3; do
ECAMD_TUNE=small_crc_dbg=$dbg timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/r06_crcdbg_$dbg -o run --output-format csv -- python3 tools/percall_trace.py 4096 300 2 > gpurun_out/r06_crcdbg_$dbg.log 2>&1 || exit 1
done
echo DBG_OK

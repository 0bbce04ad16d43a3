set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmcw
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_INSTS_SENDMSG -d gpurun_out/pmcw/a -o p --output-format csv -- python3 tools/pmc_probe.py 1000 wave 1 > gpurun_out/pmcw/a.out 2> gpurun_out/pmcw/a.err || { tail -5 gpurun_out/pmcw/a.err; exit 1; }
python3 tools/pmc_summary.py gpurun_out/pmcw/a

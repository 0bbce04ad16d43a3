set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/wgpmc
for G in 16 32; do
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_WAIT_INST_LDS -d gpurun_out/wgpmc/a$G -o p --output-format csv -- python3 tools/pmc_probe.py 1000 wg $G 2 > gpurun_out/wgpmc/a$G.out 2> gpurun_out/wgpmc/a$G.err || { tail -5 gpurun_out/wgpmc/a$G.err; exit 1; }
timeout -s KILL 60 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_ANY -d gpurun_out/wgpmc/b$G -o p --output-format csv -- python3 tools/pmc_probe.py 1000 wg $G 2 > gpurun_out/wgpmc/b$G.out 2> gpurun_out/wgpmc/b$G.err || { tail -5 gpurun_out/wgpmc/b$G.err; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/wgpmc/a16 gpurun_out/wgpmc/b16 gpurun_out/wgpmc/a32 gpurun_out/wgpmc/b32

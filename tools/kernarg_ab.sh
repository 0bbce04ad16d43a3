set -o pipefail
export TMPDIR=/tmp AB_PREHEAT_MS=300; mkdir -p gpurun_out
L=gfp_gaussian_process_amd/lib
{
timeout -k 10 60 build/diag/launch_latency || exit 1
echo "=== HIP_FORCE_DEV_KERNARG=0"
HIP_FORCE_DEV_KERNARG=0 timeout -k 10 60 build/diag/launch_latency || exit 1
for i in 1 2 3; do
 echo "--- default"; timeout -k 10 120 python tools/ab_lib.py $L auto 1000 || exit 1
 echo "--- kernarg host"; HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 python tools/ab_lib.py $L auto 1000 || exit 1
done
for i in 1 2; do
 echo "--- default ex"; timeout -k 10 120 python tools/ab_lib.py $L auto 0 || exit 1
 echo "--- kernarg host ex"; HIP_FORCE_DEV_KERNARG=0 timeout -k 10 120 python tools/ab_lib.py $L auto 0 || exit 1
done
} > gpurun_out/kernarg.txt 2>&1

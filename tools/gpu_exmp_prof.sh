#!/bin/bash
# rocprofv3 kernel trace of the reference's example command (-m -p) through the CLI: how much of
# the wall time the lookahead launches spend on the device
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/exmp_in
python3 -c "
import gzip, shutil
shutil.copyfileobj(gzip.open('tests/golden/example_input.csv.gz','rb'), open('gpurun_out/exmp_in/input.csv','wb'))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/exmp_prof -o exmp --output-format csv -- gfp_gaussian_process_amd/lib/ggp -i gpurun_out/exmp_in/input.csv -b tests/golden/example_parameter_file.txt -c tests/golden/example_csv_config.txt -m -p -g 1 -o gpurun_out/exmp_out > gpurun_out/exmp_prof.log 2>&1 || { tail -20 gpurun_out/exmp_prof.log; exit 1; }
rm -rf gpurun_out/exmp_in gpurun_out/exmp_out
f=$(find gpurun_out/exmp_prof -name "*kernel_stats*" | head -1)
cut -c1-220 "$f"

# config D shard: kernel trace with the default build and with the 2.5 KiB / 448-entry LDS build
set -o pipefail
mkdir -p gpurun_out/prof_D_a gpurun_out/prof_D_b
export TMPDIR=/tmp
timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_D_a -o t -- python3 -u bench.py --mode sharded --config D --shard-of 8 --steps 10 --warmup 2 > gpurun_out/prof_D_a/b.json 2> gpurun_out/prof_D_a/b.err || exit $?
EMQX_TM_LIB=$PWD/emqx_amd/variants/libemqx_tm_tb2560_f448.so timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_D_b -o t -- python3 -u bench.py --mode sharded --config D --shard-of 8 --steps 10 --warmup 2 > gpurun_out/prof_D_b/b.json 2> gpurun_out/prof_D_b/b.err || exit $?
cut -d, -f1-4 gpurun_out/prof_D_a/t_kernel_stats.csv | head -8; cut -d, -f1-4 gpurun_out/prof_D_b/t_kernel_stats.csv | head -8

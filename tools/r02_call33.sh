# kernel split of the flat path with and without prescan thresholds (ring scan), rocprof stats
source tools/gpu_steps.sh
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step 300 gpurun_out/r02_flat_pre0_stats.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pre0 -o run -- python tools/ab_flat.py --dims 128
export ALAYA_FLAT_PRESCAN=32
step 300 gpurun_out/r02_flat_pre32_stats.log rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_pre32 -o run -- python tools/ab_flat.py --dims 128

# random-row gather ceilings per row size (SIFT 512 B, SQ8 768 B, GIST 3840 B)
source tools/gpu_steps.sh
step 300 gpurun_out/r02_gather_probe.log ./tools/gather_probe

# round-2 secondary configs with their CPU legs, the flat config-2 line with its CPU leg, and a
# two-rank rehearsal of `bench.py --gpus 2` (both ranks on cuda:0 over gloo; code path only)
source tools/gpu_steps.sh
export TMPDIR=/tmp
# (done in an earlier call) step 500 gpurun_out/r02_sift.log python -u bench.py --workload sift-hnsw --sweep-qps --steps 20 --warmup 3
step 600 gpurun_out/r02_gist10k.log python -u bench.py --nq 10000 --steps 10 --warmup 2
step 700 gpurun_out/r02_c5.log python -u bench.py --workload sq8-ip --steps 20 --warmup 3
step 400 gpurun_out/r02_flat_c2.log python -u bench.py --workload flat --steps 20 --warmup 3
ALAYA_BENCH_REHEARSE=1 step 500 gpurun_out/r02_rehearse2.log python -u bench.py --gpus 2 --n 200000 --steps 5 --warmup 2 --no-cpu-baseline
for f in r02_gist10k r02_c5 r02_flat_c2 r02_rehearse2; do grep '^{' gpurun_out/$f.log > gpurun_out/$f.json || true; done
python - <<'PY'
import json
for f in ("r02_gist10k", "r02_c5", "r02_flat_c2", "r02_rehearse2"):
    try:
        d = json.load(open(f"gpurun_out/{f}.json"))
    except Exception as e:
        print(f, "missing", e); continue
    c = d["config"]
    print(f, d["value"], d["n_gpus"], c.get("ef_search"), c.get("recall_at_10"), d["roofline"]["kernel_ms"],
          d["roofline"]["frac"], (d["cpu_baseline"] or {}).get("value"))
PY

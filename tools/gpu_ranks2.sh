# two-rank rehearsal of the driver's N>1 bench launch on a one-GPU box (both ranks on device 0: gloo)
set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 \
    bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu --no-extras > gpurun_out/ranks2.log 2>&1 || { tail -30 gpurun_out/ranks2.log; exit 1; }
python - <<'PY'
import json
l = [x for x in open("gpurun_out/ranks2.log") if x.startswith("{")][-1]
d = json.loads(l)
print("n_gpus", d["n_gpus"], "value", round(d["value"]), "world", d.get("world_size"), "backend", d.get("collective_backend"),
      "lba ms/iter", d["lba"]["ms_per_iter"], "lba collective", d["lba"].get("collective"))
PY

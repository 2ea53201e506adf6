"""Throughput of the real product -- ``src/main_pretrain.py`` fed by loader workers from JPEG tar
shards -- against ``bench.py`` (synthetic images resident on the GPU) at the same per-GPU shape.

The reference's product is ``main_pretrain`` fed by 40 webdataset workers per TPU host
(/root/reference/src/main_pretrain.py:58-75, /root/reference/src/dataset.py:100-161).  Here: the
ViT-L/16 preset (config/pretrain/pretrain-vit-l16-224-in1k-800ep.sh flags) at 512 images per GPU
(the per-GPU batch of the 8-GPU configuration), real JPEG shards at ImageNet-like sizes
(data/jpeg_shards.py, written in parallel on first use), ``--train-loader-workers`` workers, the
device augment (workers decode and ship crop windows; RandomResizedCrop + flip on the GPU,
csrc/augment.hip) and the ``DevicePrefetcher`` side stream.  The driver logs ``perf/images_per_sec``
per log window (wall clock, host syncs included); the steady state is the mean over the windows
after ``--skip`` steps.  Then ``bench.py --batch-per-gpu B`` on the same box.

    python tools/product_rate.py --out gpurun_out/prod [--steps 60] [--batch 512] [--workers 8]
    (under rocprofv3 --kernel-trace --memory-copy-trace: --driver-only, then tools/overlap_check.py)
"""

from __future__ import annotations

import argparse
import glob
import json
import multiprocessing as mp
import os
import shutil
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

VITL = ["--mode", "pretrain", "--image_mask_ratio", "0.75", "--random-crop", "rrc", "--color-jitter", "0.0",
        "--auto-augment", "none", "--random-erasing", "0.0", "--augment-repeats", "1", "--test-crop-ratio", "0.875",
        "--mixup", "0.0", "--cutmix", "0.0", "--layers", "24", "--dim", "1024", "--heads", "16", "--labels", "0",
        "--patch-size", "16", "--image-size", "224", "--posemb", "sincos2d", "--pooling", "cls", "--dropout", "0.0",
        "--droppath", "0.0", "--dec-layers", "8", "--dec-dim", "512", "--dec-heads", "16", "--dec-posemb",
        "sincos2d", "--dec-dropout", "0.0", "--dec-droppath", "0.0", "--init-seed", "0", "--mixup-seed", "0",
        "--dropout-seed", "0", "--noise-seed", "0", "--shuffle-seed", "0", "--optimizer", "adamw",
        "--learning-rate", "1.5e-4", "--weight-decay", "0.05", "--adam-b1", "0.9", "--adam-b2", "0.95",
        "--adam-eps", "1e-8", "--lr-decay", "1.0", "--clip-grad", "0.0", "--grad-accum", "1"]


def _write_one(a):
    d, i, per_shard = a
    from jumbo_mae_tpu_amd.data.jpeg_shards import write_shards
    tmp = os.path.join(d, f".w{i}")
    write_shards(tmp, shards=1, per_shard=per_shard, classes=1000, seed=1000 + i)
    os.replace(os.path.join(tmp, "train-000000.tar"), os.path.join(d, f"train-{i:06d}.tar"))
    shutil.rmtree(tmp, ignore_errors=True)


def ensure_shards(d, shards, per_shard, procs):
    if all(os.path.exists(os.path.join(d, f"train-{i:06d}.tar")) for i in range(shards)):
        return
    os.makedirs(d, exist_ok=True)
    t0 = time.time()
    with mp.get_context("spawn").Pool(procs) as pool:
        pool.map(_write_one, [(d, i, per_shard) for i in range(shards)])
    print(f"[prod] wrote {shards} x {per_shard} JPEGs in {time.time() - t0:.1f}s", file=sys.stderr, flush=True)


def driver_cmd(a, spec, out_dir):
    return [sys.executable, "-u", os.path.join(ROOT, "src", "main_pretrain.py"), *VITL,
            "--train-dataset-shards", spec, "--train-batch-size", str(a.batch), "--train-loader-workers",
            str(a.workers), "--device-augment", "on", "--training-steps", str(a.steps), "--warmup-steps", "5",
            "--log-interval", str(a.log_interval), "--eval-interval", "0", "--output-dir", out_dir,
            "--name", "prod", "--log-file-only", "--device", "cuda"]


def driver(a, spec, out_dir, log_path):
    cmd = driver_cmd(a, spec, out_dir)
    with open(log_path, "w") as f:
        r = subprocess.run(cmd, stdout=f, stderr=subprocess.STDOUT, cwd=ROOT)
    if r.returncode:
        raise SystemExit(f"driver failed ({r.returncode}), see {log_path}")
    rows = []
    for p in glob.glob(os.path.join(out_dir, "*.jsonl")):
        with open(p) as f:
            rows += [json.loads(ln) for ln in f if ln.strip()]
    win = [r for r in rows if "perf/images_per_sec" in r and r.get("step", r.get("_step", 0)) > a.skip]
    if not win:
        raise SystemExit(f"no perf rows after step {a.skip} in {out_dir}")
    ips = [r["perf/images_per_sec"] for r in win]
    return {"windows": len(ips), "images_per_sec": sum(ips) / len(ips), "per_window": [round(x, 1) for x in ips],
            "step_ms": sum(r["perf/step_ms"] for r in win) / len(win)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/prod")
    ap.add_argument("--shards-dir", default="/tmp/jmae_prod_shards")
    ap.add_argument("--shards", type=int, default=16)
    ap.add_argument("--per-shard", type=int, default=256)
    ap.add_argument("--procs", type=int, default=16)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--skip", type=int, default=20, help="steps excluded from the steady state (warm-up, loader fill)")
    ap.add_argument("--log-interval", type=int, default=10)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--workers", type=int, default=8)
    ap.add_argument("--driver-only", action="store_true")
    ap.add_argument("--print-cmd", action="store_true",
                    help="write the shards, print the driver's argv (one per line, for rocprofv3 -- ...) and exit")
    a = ap.parse_args()
    os.makedirs(a.out, exist_ok=True)
    ensure_shards(a.shards_dir, a.shards, a.per_shard, a.procs)
    spec = os.path.join(a.shards_dir, f"train-{{000000..{a.shards - 1:06d}}}.tar")
    run_dir = os.path.join("/tmp", "jmae_prod_run")
    shutil.rmtree(run_dir, ignore_errors=True)
    if a.print_cmd:
        print("\n".join(driver_cmd(a, spec, run_dir)))
        return
    res = {"config": {"model": "ViT-L/16 jumbo-MAE (preset flags)", "per_gpu_batch": a.batch, "workers": a.workers,
                      "steps": a.steps, "skip": a.skip, "device_augment": True, "cpus": os.cpu_count(),
                      "shards": f"{a.shards} x {a.per_shard} JPEG"}}
    res["driver"] = driver(a, spec, run_dir, os.path.join(a.out, "driver.log"))
    print(json.dumps({"driver": res["driver"]}), flush=True)
    if not a.driver_only:
        cmd = [sys.executable, "-u", os.path.join(ROOT, "bench.py"), "--batch-per-gpu", str(a.batch), "--steps", "30",
               "--warmup", "5"]
        r = subprocess.run(cmd, capture_output=True, text=True, cwd=ROOT)
        if r.returncode:
            raise SystemExit("bench failed:\n" + r.stderr[-2000:])
        b = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
        res["bench"] = {"images_per_sec": b["value"], "ms_per_step": b["ms_per_step"]}
        res["driver_over_bench"] = res["driver"]["images_per_sec"] / b["value"]
    with open(os.path.join(a.out, "product_rate.json"), "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()

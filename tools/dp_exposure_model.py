"""Exposure model of the data-parallel gradient path at N GPUs: which bucket size, and all-reduce or
ZeRO-1, for the ViT-L pretraining step (parallel/ddp.py).

The model replays the REAL bucket plan of ``GradReducer`` (built on the CPU from the ViT-L Jumbo-MAE
parameter store, layer-boundary buckets, the chunked jumbo-MLP tail, ZeRO-1 sub-buckets) against a
backward-pass timeline and one RCCL stream:

* backward: the measured backward time of the per-GPU step (``--backward-ms``; 512 images per GPU
  at N = 8: ~55 ms, profiles/r5a_summary_vitl_b512.txt) split over the decoder / encoder layers in
  proportion to their FLOPs, in backward order; a bucket is ready when its last segment is final
  (the shared jumbo-MLP weights only after layer 0, in ``PARTIAL_SUB`` row chunks over the batched
  weight-gradient GEMM);
* collectives: one stream, in launch order, each starting when its bucket is ready and the previous
  one has finished.  Time of a collective on ``b`` bytes = alpha + wire bytes / busbw(b) with the
  ring wire bytes 2 (n - 1) / n b (all-reduce) or (n - 1) / n b (reduce-scatter / all-gather);
  busbw(b) = busbw_max b / (b + b_half).  The defaults (alpha 25 us, 300 GB/s, b_half 4 MiB) are
  ASSUMPTIONS for RCCL on 8 x MI355X over xGMI; ``--sweep`` replaces them with a measured
  ``tools/allreduce_bench.py --json`` sweep of the node (interpolated per size);
* optimizer: AdamW over the flat store (``--adamw-ms`` for the whole model on one GPU, 2.33 ms
  measured) per optimizer group right after that group's reduction -- on 1/N of the bytes with
  ZeRO-1, whose updated weights are then all-gathered on the same stream before the next
  forward (the bf16 shadow, 2 bytes per parameter; ``zero1-fp32gather`` = the fp32 master).
  Modes: all-reduce in fp32 / bf16 (``--reduce-dtype``), ZeRO-1 with an fp32 / bf16 reduce-scatter
  and a bf16 gather, and the round-5 fp32-gather ZeRO-1.  The bf16 staging copies are not priced.

Prints, per bucket size and mode, the number of collectives, the communication time, and the time
the step waits after its backward (exposed communication + the optimizer tail).

    python tools/dp_exposure_model.py [--world 8] [--backward-ms 55] [--bucket-mb 16,32,64,128,256]
                                      [--sweep node_sweep.json] [--json out.json]
"""

from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def load_sweep(path):
    """``collective_sweep`` rows from a tools/allreduce_bench.py --json file, a bench.py JSON line
    (the multi-GPU run's self-calibration: one row per bucket size of the real plan), or a driver
    record holding that line under "parsed"."""
    d = json.load(open(path))
    for k in ("parsed", "result"):
        if "collective_sweep" not in d and isinstance(d.get(k), dict):
            d = d[k]
    return d["collective_sweep"]


def busbw_fn(args):
    if args.sweep:
        rows = load_sweep(args.sweep)
        key = next(k for k in ("allreduce_busbw_GBs", "reduce_scatter_busbw_GBs", "all_gather_busbw_GBs")
                   if any(k in r for r in rows))
        pts = sorted((r["size_mb"] * 2**20, r[key] * 1e9) for r in rows if key in r)

        def bw(b):
            if b <= pts[0][0]:
                return pts[0][1] * b / pts[0][0]
            for (x0, y0), (x1, y1) in zip(pts, pts[1:]):
                if b <= x1:
                    return y0 + (y1 - y0) * (b - x0) / (x1 - x0)
            return pts[-1][1]
        return bw
    return lambda b: args.busbw_gbs * 1e9 * b / (b + args.b_half_mb * 2**20)


def layer_times(vc, dc, backward_ms):
    """Backward duration per unit in backward order: decoder layers 7..0, encoder layers 23..0."""
    te, td = vc.num_cls_tokens + vc.keep_len, vc.num_cls_tokens + vc.seq_patches
    enc = 2 * te * 12 * vc.dim ** 2 + 4 * te * te * vc.dim + 2 * 2 * (3 * vc.dim) * (12 * vc.dim)  # + jumbo MLP
    dec = 2 * td * 12 * dc.dec_dim ** 2 + 4 * td * td * dc.dec_dim
    units = [("dec", i, dec) for i in reversed(range(dc.dec_layers))] + [("enc", i, enc) for i in reversed(range(vc.layers))]
    tot = sum(u[2] for u in units)
    return [(k, i, backward_ms * f / tot) for k, i, f in units]


def final_times(red, vc, dc, backward_ms, parts):
    """Per segment of the reducer: the backward time (ms) at which its gradient is final, and for
    the jumbo kernels the chunk times."""
    import re
    t, fin = 0.0, {}
    for k, i, d in layer_times(vc, dc, backward_ms):
        t += d
        fin[(k, i)] = t
    jumbo_gemm = 0.03 * backward_ms  # the batched 24-layer jumbo weight-gradient GEMM (~1.6 ms at 55)
    out = []
    for s in red.segs:
        p = "/".join(s.path)
        m = re.search(r"(dec_)?layer_(\d+)", p)
        if "jumbo_mlp" in p:
            out.append(("chunks", [backward_ms + jumbo_gemm * (c + 1) / parts for c in range(parts)]))
        elif m:
            out.append(("t", fin[("dec" if m.group(1) else "enc", int(m.group(2)))]))
        elif p.startswith("decoder"):
            out.append(("t", fin[("dec", dc.dec_layers - 1)] * 0.02 if "pred" in p or "norm" in p
                        else fin[("dec", 0)]))
        else:  # encoder embedding, cls tokens, final norm
            out.append(("t", backward_ms + jumbo_gemm if "embed" in p else fin[("enc", vc.layers - 1)]))
    return out


def simulate(red, segt, world, bw, alpha_ms, adamw_ms, backward_ms, shard, opt_groups=4, rbytes=4, gbytes=2):
    """``rbytes``: bytes per element of the gradient reduction (4 fp32, 2 with --reduce-dtype bf16);
    ``gbytes``: of the ZeRO-1 weight all-gather (2: the bf16 shadow, the default; 4: the fp32
    master, the round-5 path)."""
    n = world
    elems = sum(hi - lo for lo, hi, _ in red.buckets)
    total = elems * rbytes
    ready = []
    for lo, hi, idxs in red.buckets:
        r = 0.0
        for i in idxs:
            kind, v = segt[i]
            s = red.segs[i]
            if kind == "t":
                r = max(r, v)
            else:  # chunked: the chunk covering the end of this bucket's overlap with the segment
                a, b = max(lo, s.offset) - s.offset, min(hi, s.offset + s.numel) - s.offset
                r = max(r, v[min(len(v) - 1, (b - 1) * len(v) // s.numel)])
        ready.append(r)
    # all-reduce mode launches the jumbo chunks as partial slices: model each chunk as its own piece
    pieces = []
    for (lo, hi, idxs), r in zip(red.buckets, ready):
        segs = [red.segs[i] for i in idxs]
        if not shard and len(segs) == 1 and segt[idxs[0]][0] == "chunks":
            v = segt[idxs[0]][1]
            for c, tc in enumerate(v):
                pieces.append((tc, (hi - lo) * rbytes / len(v)))
        else:
            pieces.append((r, (hi - lo) * rbytes))
    pieces.sort(key=lambda x: x[0])  # issued as they become ready (GradReducer._on_ready / _on_partial)
    fac = (n - 1) / n * (1 if shard else 2)
    t, comm, ends = 0.0, 0.0, []
    for r, b in pieces:
        d = alpha_ms + b * fac / bw(b) * 1e3
        t = max(t, r) + d
        comm += d
        ends.append(t)
    red_end = t
    # optimizer groups: consecutive equal shares of the buckets, each after its last reduction
    k = len(ends)
    groups = [ends[k * g // opt_groups: k * (g + 1) // opt_groups] for g in range(opt_groups)]
    upd_ms = adamw_ms / (n if shard else 1) / opt_groups
    comp = backward_ms
    gather_t = red_end
    for g in groups:
        if not g:
            continue
        comp = max(comp, g[-1]) + upd_ms
        if shard:  # all-gather of the group's updated weights (bf16 shadow / fp32 master), same RCCL stream
            gb = elems * gbytes / opt_groups
            d = alpha_ms + gb * (n - 1) / n / bw(gb) * 1e3
            gather_t = max(gather_t, comp) + d
            comm += d
    step_end = max(comp, gather_t if shard else red_end)
    return {"collectives": len(pieces) + (opt_groups if shard else 0), "comm_ms": round(comm, 3),
            "reduce_done_after_backward_ms": round(max(0.0, red_end - backward_ms), 3),
            "wait_after_backward_ms": round(step_end - backward_ms, 3)}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--backward-ms", type=float, default=55.0)
    ap.add_argument("--adamw-ms", type=float, default=2.33)
    ap.add_argument("--bucket-mb", default="8,16,32,64,128,256")
    ap.add_argument("--busbw-gbs", type=float, default=300.0)
    ap.add_argument("--b-half-mb", type=float, default=4.0)
    ap.add_argument("--alpha-us", type=float, default=25.0)
    ap.add_argument("--sweep", default="")
    ap.add_argument("--json", default="")
    a = ap.parse_args(argv)
    import torch
    from jumbo_mae_tpu_amd.config import decoder_config, vit_config
    from jumbo_mae_tpu_amd.models.mae import PretrainModel
    from jumbo_mae_tpu_amd.models import params as PM
    from jumbo_mae_tpu_amd.parallel import ddp

    vc = vit_config("vit_large_patch16", labels=0, posemb="sincos2d", image_mask_ratio=0.75)
    dc = decoder_config()
    # the bucket plan only needs segment offsets: skip the 405 M-parameter initialisation
    orig = PM.ParamStore.initialize
    PM.ParamStore.initialize = lambda self, generator=None: None
    try:
        store = PretrainModel(vc, dc).to("cpu", torch.float32, seed=0).store
    finally:
        PM.ParamStore.initialize = orig
    q = a.world * PM.ALIGN
    store.total = -(-store.total // q) * q
    bw = busbw_fn(a)
    rows = []
    variants = [("all-reduce", False, 4, 0), ("all-reduce-bf16", False, 2, 0), ("zero1", True, 4, 2),
                ("zero1-bf16", True, 2, 2), ("zero1-fp32gather", True, 4, 4)]
    for mb in [float(x) for x in a.bucket_mb.split(",")]:
        for mode, shard, rb, gbb in variants:
            red = ddp.GradReducer(store, bucket_mb=mb)
            if shard:  # the ZeRO-1 plan (ddp.GradReducer shard=True) without a process group
                limit = int(mb * 2**20 / 4)
                rngs = ddp.shard_ranges([(lo, hi) for lo, hi, _ in red.buckets], q)
                rngs = ddp.split_oversized(rngs, [(s.offset, s.numel) for s in red.segs if s.numel > limit], q)
                red.buckets = [(lo, hi, [i for i, s in enumerate(red.segs) if s.offset < hi and s.offset + s.numel > lo])
                               for lo, hi in rngs]
            segt = final_times(red, vc, dc, a.backward_ms, ddp.PARTIAL_SUB)
            r = simulate(red, segt, a.world, bw, a.alpha_us / 1e3, a.adamw_ms, a.backward_ms, shard,
                         rbytes=rb, gbytes=gbb)
            r.update({"bucket_mb": mb, "mode": mode, "buckets": len(red.buckets)})
            rows.append(r)
            print(f"bucket {mb:6.1f} MB  {r['mode']:16s}  buckets {r['buckets']:3d}  collectives {r['collectives']:3d}  "
                  f"comm {r['comm_ms']:7.2f} ms  reductions end +{r['reduce_done_after_backward_ms']:.2f} ms  "
                  f"step waits +{r['wait_after_backward_ms']:.2f} ms after the backward")
    best = min(rows, key=lambda r: (r["wait_after_backward_ms"], r["collectives"]))
    out = {"world": a.world, "backward_ms": a.backward_ms,
           "assumptions": {"busbw_GBs": a.busbw_gbs, "b_half_mb": a.b_half_mb, "alpha_us": a.alpha_us,
                           "sweep": a.sweep or None},
           "rows": rows, "best": best}
    print(json.dumps({"best": best}))
    if a.json:
        json.dump(out, open(a.json, "w"), indent=1)


if __name__ == "__main__":
    main()

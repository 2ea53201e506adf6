"""Shard-reading throughput: native reader (jumbo_mae_tpu_amd._io, C++ threads, ordered read-ahead)
vs the Python tarfile reader (data/shards.py tar_samples), on synthetic ImageNet-like shards
(~110 KB "jpg" + "cls" per sample) written to a temp dir.

    python tools/io_bench.py --shards 16 --per-shard 200 --threads 1,4,8
"""

import argparse
import io
import os
import sys
import tarfile
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from jumbo_mae_tpu_amd.data import shards as S  # noqa: E402


def make(d, shards, per, kb):
    urls = []
    for s in range(shards):
        p = os.path.join(d, f"shard-{s:04d}.tar")
        with tarfile.open(p, "w") as tf:
            for i in range(per):
                for ext, data in (("jpg", os.urandom(kb * 1024)), ("cls", str(i % 1000).encode())):
                    ti = tarfile.TarInfo(f"{s:04d}_{i:06d}.{ext}")
                    ti.size = len(data)
                    tf.addfile(ti, io.BytesIO(data))
        urls.append(p)
    return urls


def rate(fn, nbytes):
    t = time.perf_counter()
    n = sum(1 for _ in fn())
    dt = time.perf_counter() - t
    return n, n / dt, nbytes / dt / 1e6


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shards", type=int, default=16)
    ap.add_argument("--per-shard", type=int, default=200)
    ap.add_argument("--kb", type=int, default=110)
    ap.add_argument("--threads", default="1,4,8")
    a = ap.parse_args()
    from jumbo_mae_tpu_amd import _io
    with tempfile.TemporaryDirectory() as d:
        urls = make(d, a.shards, a.per_shard, a.kb)
        nbytes = sum(os.path.getsize(u) for u in urls)
        for u in urls:  # page cache warm for both readers
            open(u, "rb").read()
        n, sps, mbs = rate(lambda: (s for u in urls for s in S.tar_samples(u)), nbytes)
        print(f"python tarfile          {n} samples  {sps:9.0f} samples/s  {mbs:8.0f} MB/s", flush=True)
        for t in (int(x) for x in a.threads.split(",")):
            n, sps, mbs = rate(lambda: _io.ShardReader(urls, threads=t), nbytes)
            print(f"native threads={t:<2d}      {n} samples  {sps:9.0f} samples/s  {mbs:8.0f} MB/s", flush=True)


if __name__ == "__main__":
    main()

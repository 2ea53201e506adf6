"""webdataset-compatible shard reading (webdataset is not installed here).

Reference pipeline (/root/reference/src/dataset.py:107-116,139-150):
  SimpleShardList(urls, seed) -> cycle -> detshuffle -> slice(rank, None, world)
  -> split_by_worker -> tarfile_to_samples(ignore_and_continue) -> detshuffle -> decode
Implemented here with the stdlib ``tarfile`` in streaming mode: brace-expanded shard lists,
deterministic per-epoch shard shuffles, rank/worker splitting, sample grouping by key
(``{key}.jpg`` + ``{key}.cls`` -> one sample), a deterministic shuffle buffer, and
``pipe:`` URLs (e.g. ``pipe:gsutil cat gs://...``) next to local files.

Local shards are read by the native module ``jumbo_mae_tpu_amd._io`` when it is built
(csrc/io/tario.cpp: tar parsing and file I/O on a pool of C++ threads with ordered read-ahead, the
same sample stream as the Python reader); ``JMAE_NATIVE_IO=0`` forces the Python path.
"""

from __future__ import annotations

import io
import itertools
import os
import random
import re
import subprocess
import tarfile
from typing import Iterable, Iterator


def brace_expand(pattern: str) -> list[str]:
    """'a-{000..002}.tar' -> ['a-000.tar','a-001.tar','a-002.tar']; also {a,b} alternatives."""
    m = re.search(r"\{([^{}]*)\}", pattern)
    if not m:
        return [pattern]
    body = m.group(1)
    pre, post = pattern[:m.start()], pattern[m.end():]
    rng = re.fullmatch(r"(\d+)\.\.(\d+)", body)
    if rng:
        a, b = rng.group(1), rng.group(2)
        width = len(a)
        items = [str(i).zfill(width) for i in range(int(a), int(b) + 1)]
    else:
        items = body.split(",")
    out = []
    for it in items:
        out.extend(brace_expand(pre + it + post))
    return out


def shard_list(spec: str | list[str]) -> list[str]:
    if isinstance(spec, (list, tuple)):
        return [u for s in spec for u in shard_list(s)]
    urls = []
    for part in spec.split("::"):
        urls.extend(brace_expand(part))
    return urls


def open_stream(url: str):
    if url.startswith("pipe:"):
        p = subprocess.Popen(url[5:], shell=True, stdout=subprocess.PIPE)
        return p.stdout
    if url.startswith("file://"):
        url = url[7:]
    return open(url, "rb")


def _split_key(name: str) -> tuple[str, str]:
    base = name.rsplit("/", 1)[-1]
    if "." not in base:
        return name, ""
    i = name.rfind("/") + 1 + base.index(".")
    return name[:i], name[i + 1:]


def tar_samples(url: str, handler=None) -> Iterator[dict]:
    """Yield {'__key__', '__url__', ext: bytes} groups from one tar shard."""
    try:
        with open_stream(url) as f, tarfile.open(fileobj=f, mode="r|*") as tf:
            cur: dict | None = None
            for ti in tf:
                if not ti.isreg():
                    continue
                key, ext = _split_key(ti.name)
                if not ext:
                    continue
                data = tf.extractfile(ti).read()
                if cur is None or cur["__key__"] != key:
                    if cur is not None:
                        yield cur
                    cur = {"__key__": key, "__url__": url}
                cur[ext.lower()] = data
            if cur is not None:
                yield cur
    except Exception as e:  # ignore_and_continue semantics
        if handler is None:
            raise
        handler(e)


def _native():
    if os.environ.get("JMAE_NATIVE_IO", "1") != "1":
        return None
    try:
        from .. import _io
    except ImportError:
        return None
    return _io


def _local_path(url: str) -> str | None:
    if url.startswith("pipe:"):
        return None
    return url[7:] if url.startswith("file://") else url


def iter_samples(urls: list[str], handler=None, threads: int = 4) -> Iterator[dict]:
    """Samples of several shards in order: ``chain(tar_samples(u, handler) for u in urls)``.

    With the native reader every local shard is parsed by a C++ thread pool (``threads`` shards in
    flight, samples handed out in shard order); a shard error is skipped when ``handler`` is given
    (ignore_and_continue) and raised otherwise, after the samples read before the fault."""
    nat = _native()
    paths = [_local_path(u) for u in urls]
    if nat is None or not urls or any(p is None for p in paths):
        yield from itertools.chain.from_iterable(tar_samples(u, handler) for u in urls)
        return
    url_of = dict(zip(paths, urls))  # report the URL as given (file:// prefix kept)
    reader = nat.ShardReader(paths, threads=threads, ignore_errors=handler is not None)
    try:
        for s in reader:
            s["__url__"] = url_of.get(s["__url__"], s["__url__"])
            yield s
    except RuntimeError as e:
        if handler is None:
            raise
        handler(e)
    finally:
        reader.close()


def ignore_and_continue(exn) -> bool:
    return True


def detshuffle(items: Iterable, bufsize: int, seed: int) -> Iterator:
    """Deterministic buffered shuffle (webdataset detshuffle)."""
    rng = random.Random(seed)
    buf = []
    for x in items:
        buf.append(x)
        if len(buf) >= bufsize:
            i = rng.randrange(len(buf))
            buf[i], buf[-1] = buf[-1], buf[i]
            yield buf.pop()
    rng.shuffle(buf)
    yield from buf


def epoch_shards(urls: list[str], seed: int, epoch: int, shuffle: bool) -> list[str]:
    urls = list(urls)
    if shuffle:
        random.Random(seed * 1000003 + epoch).shuffle(urls)
    return urls


def split(urls: list[str], index: int, count: int) -> list[str]:
    return list(itertools.islice(urls, index, None, count))


def decode_pil(data: bytes):
    from PIL import Image

    img = Image.open(io.BytesIO(data))
    img.load()
    return img.convert("RGB")


def decode_cls(data: bytes) -> int:
    return int(data.decode().strip())

"""webdataset-compatible shard reading (webdataset is not installed here).

Reference pipeline (/root/reference/src/dataset.py:107-116,139-150):
  SimpleShardList(urls, seed) -> cycle -> detshuffle -> slice(rank, None, world)
  -> split_by_worker -> tarfile_to_samples(ignore_and_continue) -> detshuffle -> decode
Implemented here with the stdlib ``tarfile`` in streaming mode: brace-expanded shard lists,
deterministic per-epoch shard shuffles, rank/worker splitting, sample grouping by key
(``{key}.jpg`` + ``{key}.cls`` -> one sample), a deterministic shuffle buffer, and
``pipe:`` / ``gs://`` / ``s3://`` / ``http(s)://`` URLs next to local files (utils/gopen.py; the
reference's presets read ``$GCS_DATASET_DIR`` = ``gs://...`` through webdataset's gopen).

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

from ..utils import gopen


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


class PipeStream(io.RawIOBase):
    """stdout of a ``pipe:`` command; ``close`` reaps the command and raises ``IOError`` when it
    failed, so a truncated download is an error rather than a silently short shard.  A command
    killed by SIGPIPE because the reader stopped early is not an error."""

    def __init__(self, cmd: str):
        self.cmd = cmd
        self.proc = subprocess.Popen(cmd, shell=True, stdout=subprocess.PIPE)
        self._eof = False

    def readable(self):
        return True

    def readinto(self, b):
        n = self.proc.stdout.readinto(b)
        if not n:
            self._eof = True
        return n

    def close(self):
        if self.closed:
            return
        self.proc.stdout.close()
        rc = self.proc.wait()
        super().close()
        if rc != 0 and not (not self._eof and rc in (-13, 141)):
            raise IOError(f"pipe command failed with exit status {rc}: {self.cmd}")


def open_stream(url: str):
    """Byte stream of a shard: local file, or the stdout of the scheme's read command (``pipe:``,
    ``gs://`` via gsutil, ``s3://``, ``http(s)://`` via curl -- utils/gopen.py)."""
    local = gopen.local_path(url)
    if local is not None:
        return open(local, "rb")
    return io.BufferedReader(PipeStream(gopen.command(url, "read")), 1 << 20)


def cache_dir() -> str:
    """Shard cache directory: ``$WDS_CACHE`` or ``./_cache`` (webdataset's defaults)."""
    return os.environ.get("WDS_CACHE", "./_cache")


def cache_name(url: str) -> str:
    """File name of a cached shard: the basename of the last word of the URL (the object a
    ``pipe:gsutil cat gs://bucket/val-0003.tar`` command streams) behind a short hash of the whole
    URL, so equal basenames from different buckets do not collide."""
    import hashlib

    target = url[5:].split()[-1] if url.startswith("pipe:") else url.split("?", 1)[0]
    base = re.sub(r"[^\w.\-]", "_", target.rstrip("/").rsplit("/", 1)[-1]) or "shard"
    return hashlib.sha1(url.encode()).hexdigest()[:10] + "-" + base


def cached_path(url: str, directory: str | None = None) -> str:
    """Local path of ``url``, streaming a remote/``pipe:`` shard into the cache once.

    Equivalent of webdataset's ``cached_tarfile_to_samples`` download step used by the reference
    validation pipeline (/root/reference/src/dataset.py:139-150): the first pass over the
    validation set streams each shard to ``<cache>/<name>`` (written to a temporary file and
    renamed into place, so a concurrent worker or an interrupted download never leaves a partial
    shard under the final name; the command's exit status is checked), later passes read the
    local copy.  Local files are read in place."""
    local = _local_path(url)
    if local is not None:
        return local
    directory = directory or cache_dir()
    os.makedirs(directory, exist_ok=True)
    dest = os.path.join(directory, cache_name(url))
    if os.path.exists(dest):
        return dest
    tmp = f"{dest}.{os.getpid()}.tmp"
    try:
        with open_stream(url) as src, open(tmp, "wb") as out:
            while True:
                buf = src.read(1 << 22)
                if not buf:
                    break
                out.write(buf)
        os.replace(tmp, dest)
    finally:
        if os.path.exists(tmp):
            os.unlink(tmp)
    return dest


def cached_samples(urls: list[str], handler=None, directory: str | None = None) -> Iterator[dict]:
    """``iter_samples`` over the cached copies of ``urls``; each shard is fetched when the stream
    reaches it (a failed fetch goes to ``handler`` like a read error)."""
    for u in urls:
        try:
            p = cached_path(u, directory)
        except Exception as e:
            if handler is None:
                raise
            handler(e)
            continue
        for smp in iter_samples([p], handler):
            smp["__url__"] = u
            yield smp


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


_local_path = gopen.local_path


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
    return img if img.mode == "RGB" else img.convert("RGB")  # (convert would copy an RGB image)


def decode_cls(data: bytes) -> int:
    return int(data.decode().strip())

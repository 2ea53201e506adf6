"""URL-scheme dispatch for every file the framework reads or writes (shards, checkpoints, resume
sidecars, pretrained parameters): the role ``webdataset.gopen`` plays in the reference.

Reference call sites (/root/reference):
  src/utils.py:55-63 ........ checkpoint write ``wds.gopen(f"{output_dir}/{name}-{postfix}.msgpack", "wb")``
  src/utils.py:151 .......... pretrained read ``wds.gopen(args.pretrained_ckpt)``
  src/dataset.py:107-116 .... shard streams (``tarfile_to_samples`` -> gopen)
  config/ft.sh:3-6 .......... every preset passes ``$GCS_DATASET_DIR/...`` = ``gs://...``

Schemes (webdataset's defaults, as shell commands whose stdin/stdout carry the bytes):
  local path / ``file://``  plain file IO
  ``pipe:<cmd>``            read: stdout of ``cmd``; write: ``cmd`` gets the bytes on stdin
  ``gs://``                 read ``gsutil cat <url>``; write ``gsutil cp - <url>``; exists ``gsutil -q stat``
  ``s3://``                 read ``aws s3 cp <url> -``; write ``aws s3 cp - <url>``; exists ``aws s3 ls``
  ``http(s)://``            read ``curl -fsSL <url>`` (read-only); exists ``curl -fsIL``
The command templates can be overridden with ``JMAE_GOPEN_<SCHEME>_{READ,WRITE,STAT}``
(``{url}`` is substituted, shell-quoted), e.g. ``JMAE_GOPEN_GS_READ='gcloud storage cat {url}'``.
"""

from __future__ import annotations

import os
import shlex
import subprocess

_DEFAULTS = {
    "gs": {"read": "gsutil cat {url}", "write": "gsutil cp - {url}", "stat": "gsutil -q stat {url}"},
    "s3": {"read": "aws s3 cp {url} -", "write": "aws s3 cp - {url}", "stat": "aws s3 ls {url}"},
    "http": {"read": "curl -fsSL {url}", "write": None, "stat": "curl -fsIL -o /dev/null {url}"},
    "https": {"read": "curl -fsSL {url}", "write": None, "stat": "curl -fsIL -o /dev/null {url}"},
}


def scheme(url: str) -> str:
    """'' for local paths (and ``file://``), 'pipe' for ``pipe:`` commands, else the URL scheme."""
    if url.startswith("pipe:"):
        return "pipe"
    i = url.find("://")
    if i <= 0:
        return ""
    s = url[:i].lower()
    return "" if s == "file" else s


def is_local(url: str) -> bool:
    return scheme(url) == ""


def local_path(url: str) -> str | None:
    """The filesystem path of a local URL, None for anything that needs a command."""
    if not is_local(url):
        return None
    return url[7:] if url.startswith("file://") else url


def command(url: str, op: str) -> str:
    """Shell command that performs ``op`` ('read' | 'write' | 'stat') on a non-local URL."""
    s = scheme(url)
    if s == "pipe":
        if op == "stat":
            raise ValueError(f"cannot test existence of a pipe: URL: {url}")
        return url[5:]
    if s not in _DEFAULTS:
        raise ValueError(f"unsupported URL scheme {s!r}: {url}")
    tmpl = os.environ.get(f"JMAE_GOPEN_{s.upper()}_{op.upper()}") or _DEFAULTS[s][op]
    if tmpl is None:
        raise ValueError(f"{s}:// URLs are read-only ({op} requested): {url}")
    return tmpl.replace("{url}", shlex.quote(url))


def join(base: str, *parts: str) -> str:
    """``os.path.join`` for local paths, '/'-join for URLs (never turns ``gs://b`` into ``gs:/b``)."""
    if is_local(base):
        return os.path.join(base, *parts)
    if scheme(base) == "pipe":
        raise ValueError(f"cannot join a path onto a pipe: command: {base}")
    out = base
    for p in parts:
        out = out.rstrip("/") + "/" + p.lstrip("/")
    return out


def read_bytes(url: str) -> bytes:
    p = local_path(url)
    if p is not None:
        with open(p, "rb") as f:
            return f.read()
    return subprocess.run(command(url, "read"), shell=True, check=True, capture_output=True).stdout


def write_bytes(url: str, data: bytes) -> None:
    """Local: write to a temporary file, fsync, atomic rename.  Remote / ``pipe:``: the bytes go to
    the scheme's write command on stdin; a non-zero exit status raises."""
    p = local_path(url)
    if p is None:
        subprocess.run(command(url, "write"), shell=True, check=True, input=data)
        return
    d = os.path.dirname(p)
    if d:
        os.makedirs(d, exist_ok=True)
    tmp = f"{p}.tmp.{os.getpid()}"
    with open(tmp, "wb") as f:
        f.write(data)
        f.flush()
        os.fsync(f.fileno())
    os.replace(tmp, p)


def exists(url: str) -> bool:
    p = local_path(url)
    if p is not None:
        return os.path.exists(p)
    r = subprocess.run(command(url, "stat"), shell=True, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    return r.returncode == 0

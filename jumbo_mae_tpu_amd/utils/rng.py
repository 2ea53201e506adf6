"""Per-rank random streams: ``mixup``, ``dropout``, ``noise``.

Reference: TrainState keeps three PRNG keys seeded with ``seed + process_index`` and gives every
device its own sub-key (``shard_prng_key``), advancing them every step with ``split_rngs``
(/root/reference/src/pretraining.py:50-73,264-266).  Here every GPU is its own process, so
each stream is a device ``torch.Generator`` seeded from (stream seed, global rank); draws advance
the Philox offset, which is what keeps steps distinct.  Bitwise parity with JAX's threefry is
not reproducible ("parity unpinned"); the statistical contract (independent per rank, per
stream, per step, deterministic for a given seed) is.
"""

from __future__ import annotations

import hashlib

import torch

STREAMS = ("mixup", "dropout", "noise")


def derive_seed(seed: int, stream: str, rank: int) -> int:
    h = hashlib.sha256(f"{seed}:{stream}:{rank}".encode()).digest()
    return int.from_bytes(h[:8], "little") & ((1 << 63) - 1)


class RngStreams:
    def __init__(self, seeds: dict[str, int], rank: int, device):
        self.seeds = dict(seeds)
        self.rank = rank
        self.device = torch.device(device)
        self.gens = {}
        for name in STREAMS:
            g = torch.Generator(device=self.device)
            g.manual_seed(derive_seed(self.seeds.get(name, 0), name, rank))
            self.gens[name] = g

    def get(self, name: str) -> torch.Generator:
        return self.gens[name]

    def as_dict(self) -> dict[str, torch.Generator]:
        return dict(self.gens)

    def state_dict(self) -> dict:
        return {k: g.get_state() for k, g in self.gens.items()}

    def reseed(self, step: int) -> None:
        """Streams keyed by (seed, stream, rank, step): used on a resume whose saved per-rank
        states do not match this world size."""
        for name, g in self.gens.items():
            g.manual_seed(derive_seed(self.seeds.get(name, 0) * 1_000_003 + step, name, self.rank))

    def fork(self) -> "RngStreams":
        """Streams that start at this object's current states and never advance it.  Validation
        draws from a fork: the reference's validation_step splits the state's keys and drops the
        update (/root/reference/src/pretraining.py:162-167), so evaluating never moves the training
        streams -- and an interrupted run resumes exactly whether or not its save step evaluated."""
        new = RngStreams.__new__(RngStreams)
        new.seeds, new.rank, new.device = dict(self.seeds), self.rank, self.device
        new.gens = {}
        for k, g in self.gens.items():
            ng = torch.Generator(device=self.device)
            ng.set_state(g.get_state())
            new.gens[k] = ng
        return new

    def load_state_dict(self, d: dict) -> None:
        for k, s in d.items():
            if k in self.gens:
                self.gens[k].set_state(s)

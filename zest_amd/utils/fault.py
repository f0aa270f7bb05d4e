"""Fault-injection spec shared by the native server (ZEST_FAULT / `zest serve --fault`) and the
Python fakes: "drop:0.1,corrupt:0.05,delay:20" (probabilities per request, delay in ms)."""
from __future__ import annotations

import os
import random
from dataclasses import dataclass


@dataclass
class FaultSpec:
    drop: float = 0.0
    corrupt: float = 0.0
    delay_ms: int = 0

    @classmethod
    def parse(cls, s: str | None) -> "FaultSpec":
        f = cls()
        for part in (s or "").split(","):
            if not part.strip():
                continue
            k, _, v = part.partition(":")
            k = k.strip()
            if k == "drop":
                f.drop = float(v)
            elif k == "corrupt":
                f.corrupt = float(v)
            elif k == "delay":
                f.delay_ms = int(v)
            else:
                raise ValueError(f"unknown fault '{k}'")
        return f

    @classmethod
    def from_env(cls) -> "FaultSpec":
        return cls.parse(os.environ.get("ZEST_FAULT"))

    def __str__(self) -> str:
        return f"drop:{self.drop},corrupt:{self.corrupt},delay:{self.delay_ms}"

    def should_drop(self, rng=random) -> bool:
        return self.drop > 0 and rng.random() < self.drop

    def maybe_corrupt(self, data: bytes, rng=random) -> bytes:
        if self.corrupt > 0 and data and rng.random() < self.corrupt:
            b = bytearray(data)
            b[len(b) // 2] ^= 0x5A
            return bytes(b)
        return data

"""Byte-balanced contiguous split of a term table, shared by every component that has to agree on
it: the bench engine's per-rank origin shares (zest_amd.engine.plan_rank_terms) and swarm_pull's
owners when nothing is held (assign_owners).  Integer arithmetic: the two used float formulas that
could round a cut to a different side of a term boundary sitting exactly on r/N of the total -- the
8-rank rehearsal then asked a rank's memory CAS for a term another rank held (profiles/r5/
rehearsal_n8_r5am.log)."""
from __future__ import annotations

import numpy as np


def even_bounds(ulen, n: int) -> list[int]:
    """n + 1 term indices: share r is terms [b[r], b[r + 1]), ending after the first term whose
    cumulative size reaches r/n of the total (ceil(total * r / n) bytes)."""
    cu = np.cumsum(np.asarray(ulen, dtype=np.int64))
    nt = len(cu)
    total = int(cu[-1]) if nt else 0
    b = [0] + [int(np.searchsorted(cu, -(-total * r // n), side="left")) + 1 for r in range(1, n)] + [nt]
    b = np.maximum.accumulate(np.minimum(np.array(b, dtype=np.int64), nt))
    return [int(x) for x in b]

"""Golden digests of full-size merges, computed HERE with the C oracle (oracle/compose_ref.c,
itself pinned to the reference's golden vectors), for the GPU test at BASELINE sizes
(tests/test_gpu_full.py), where running the oracle would take most of a minute.

    python tools/make_full_digest.py [c3 c5 ...]  -> tests/golden/full_digests.json

Digest = sha256 over the little-endian bytes of order, addr, file, ctx and the conflict
pairs, in that order; also the output and conflict counts."""
import hashlib
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT = os.path.join(REPO, "tests", "golden", "full_digests.json")


def digest(res) -> str:
    h = hashlib.sha256()
    for a in res:
        h.update(np.ascontiguousarray(a, dtype=np.int32).tobytes())
    return h.hexdigest()


def main():
    from oracle import oracle
    from semantic_merge_amd import synth
    names = sys.argv[1:] or ["c3", "c5"]
    recs = {}
    if os.path.exists(OUT):
        recs = {r["name"]: r for r in json.load(open(OUT))}
    for name in names:
        t0 = time.time()
        soa = synth.lift_soa(synth.lift_logs(synth.CONFIGS[name]))
        t1 = time.time()
        res = oracle.compose(soa)
        t2 = time.time()
        recs[name] = {"name": name, "n_ops": int(soa.n), "n_out": int(len(res[0])),
                      "n_conflicts": int(len(res[4])), "sha256": digest(res)}
        print(f"{name}: gen {t1 - t0:.1f}s oracle {t2 - t1:.1f}s -> {recs[name]}", flush=True)
        del soa, res
    with open(OUT, "w") as f:
        json.dump(sorted(recs.values(), key=lambda r: r["name"]), f, indent=1)


if __name__ == "__main__":
    main()

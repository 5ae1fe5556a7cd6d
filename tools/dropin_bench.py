"""End-to-end cost of the drop-in ``compose_oplogs(List[Op], List[Op])`` (BASELINE config 2
shape: a synthetic two-branch lift log), split into its host and device parts.

    python tools/dropin_bench.py [--sizes 1000,10000,1000000] [--ref] [--gpu] [--out FILE]

Legs (seconds, median of --reps):
  python_from_dict / native_from_dicts  decoding the worker's op dicts into Op objects
                                        (Op.from_dict per op vs oplog.ops_from_dicts)
  json_python / json_native_pair        both branch logs' JSON texts -> Op lists + SoA: json.loads +
                                        Op.from_dict + marshal vs oplog.decode_pair (one native pass)
  python_marshal / python_materialize   the Python restatement (marshal.py, materialize.py)
  native_marshal / native_materialize   csrc/smx_host.cpp (what compose_oplogs runs)
  gpu_compose                           compose_soa on cuda:0, SoA already on the host (--gpu),
                                        split into pack (columns -> pinned staging), device
                                        (copy in, smx_compose, copy out) and unpack
  dropin_total                          compose_oplogs end to end (--gpu)
  reference_compose                     the reference's own compose_oplogs (--ref; needs
                                        /root/reference, i.e. only in the build container)
Outputs of every leg are checked equal to each other before timing is reported.
"""
from __future__ import annotations

import argparse
import gc
import json
import os
import statistics
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))

from semantic_merge_amd import synth  # noqa: E402
from semantic_merge_amd.marshal import marshal, marshal_native  # noqa: E402
from semantic_merge_amd.materialize import materialize_ops, materialize_ops_native  # noqa: E402
from semantic_merge_amd.ops import Op  # noqa: E402


def timed(fn, reps):
    ts, out = [], None
    for _ in range(reps):
        gc.collect()
        t = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t)
    return statistics.median(ts), out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sizes", default="1000000", help="total ops over both branches, comma-separated")
    ap.add_argument("--n-sym", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--ref", action="store_true")
    ap.add_argument("--gpu", action="store_true")
    ap.add_argument("--out")
    a = ap.parse_args()
    lines = []
    for n in (int(x) for x in a.sizes.split(",")):
        lines.append(one(a, n))
        print(lines[-1], flush=True)
    if a.out:
        with open(a.out, "w") as fh:
            fh.write("\n".join(lines) + "\n")


def one(a, n_ops):
    reps = a.reps if n_ops >= 100_000 else max(a.reps, 20)
    logs = synth.lift_logs(synth.LiftSpec(n_ops, min(a.n_sym, max(n_ops // 10, 10)), 11))
    A, B = synth.lift_op_dicts(logs)
    res = {"n_ops": len(A) + len(B), "reps": reps}
    res["python_from_dict"], (oa, ob) = timed(
        lambda: ([Op.from_dict(d) for d in A], [Op.from_dict(d) for d in B]), reps)
    from semantic_merge_amd.oplog import ops_from_dicts
    res["native_from_dicts"], (na_, nb_) = timed(lambda: (ops_from_dicts(A), ops_from_dicts(B)), reps)
    assert na_ == oa and nb_ == ob
    del na_, nb_
    ops = oa + ob
    ta, tb = json.dumps(A), json.dumps(B)
    res["json_python"], _ = timed(lambda: marshal([Op.from_dict(d) for d in json.loads(ta)],
                                                  [Op.from_dict(d) for d in json.loads(tb)]), reps)
    from semantic_merge_amd.oplog import decode_pair
    res["json_native_pair"], (ja, jb, jsoa) = timed(lambda: decode_pair(ta, tb), reps)
    assert ja == oa and jb == ob
    del ja, jb, jsoa

    res["python_marshal"], soa = timed(lambda: marshal(oa, ob), reps)
    res["native_marshal"], soa_n = timed(lambda: marshal_native(oa, ob), reps)
    assert all((x == y).all() for x, y in zip((soa.kind, soa.ts, soa.oid_hi, soa.oid_lo, soa.sym, soa.v0, soa.v1),
                                               (soa_n.kind, soa_n.ts, soa_n.oid_hi, soa_n.oid_lo, soa_n.sym,
                                                soa_n.v0, soa_n.v1)))
    if a.gpu:
        from semantic_merge_amd._lib import compose_soa, session
        compose_soa(soa, "cuda:0")
        splits = []

        def gpu_leg():
            out = compose_soa(soa, "cuda:0")
            splits.append(session("cuda:0").last)
            return out
        res["gpu_compose"], got = timed(gpu_leg, reps)
        for k in ("pack_s", "device_s", "unpack_s"):
            res["gpu_" + k] = statistics.median(x[k] for x in splits)
    else:
        from oracle import oracle  # test infrastructure: results to materialise when no GPU
        got = oracle.compose(soa)
    order, addr, file, ctx, pairs = got
    res["python_materialize"], out_p = timed(
        lambda: materialize_ops(ops, soa.kind, soa.strings, order, addr, file, ctx), reps)
    res["native_materialize"], out_n = timed(
        lambda: materialize_ops_native(ops, soa.kind, soa.strings, order, addr, file, ctx), reps)
    assert len(out_p) == len(out_n) and all(x == y for x, y in zip(out_p, out_n))
    del out_p
    if a.gpu:
        from semantic_merge_amd.compose import compose_oplogs
        res["dropin_total"], (out_d, conf_d) = timed(lambda: compose_oplogs(oa, ob), reps)
        assert out_d == out_n
    if a.ref:
        sys.path.insert(0, HERE)
        sys.dont_write_bytecode = True
        from make_golden import _import_reference
        rcompose, _, rops = _import_reference()
        ra = [rops.Op.from_dict(d) for d in A]
        rb = [rops.Op.from_dict(d) for d in B]
        res["reference_compose"], (out_r, conf_r) = timed(lambda: rcompose.compose_oplogs(ra, rb), 1)
        assert [o.to_dict() for o in out_r] == [o.to_dict() for o in out_n]
    return json.dumps({k: (round(v, 6) if isinstance(v, float) else v) for k, v in res.items()})


if __name__ == "__main__":
    main()

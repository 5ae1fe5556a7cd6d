"""smx_compose_async / smx_compose_finish: the host-sync-free half of a composition
(captured in a HIP graph and replayed) completes to the oracle's results
(/root/reference/semmerge/compose.py:11-114 restated in oracle/compose_ref.c)."""
import numpy as np
import pytest

from oracle import oracle
from semantic_merge_amd import _lib, synth

pytestmark = pytest.mark.gpu


def _lift(n, n_sym, seed, **kw):
    return synth.lift_soa(synth.lift_logs(synth.LiftSpec(n, n_sym, seed, **kw)))


def _check(dc, soa, label):
    got, ref = dc.results(), oracle.compose(soa)
    for name, g, r in zip(("order", "addr", "file", "ctx", "conflicts"), got, ref):
        assert np.array_equal(g, r), f"{label}: {name}"


def test_async_then_finish_matches_oracle():
    soa = _lift(200_000, 5_000, 3)
    dc = _lib.DeviceCompose(soa)
    dc.run_async()
    dc.torch.cuda.synchronize()
    assert int(dc.counts[0].item()) >= 0  # presorted plan, no None-value moves: complete
    dc.finish()
    _check(dc, soa, "async")
    assert dc.last_plan() == "presorted"


def test_async_captured_in_a_graph():
    import torch
    soa = _lift(50_000, 2_000, 4)
    dc = _lib.DeviceCompose(soa)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        dc.run_async()  # warm up (first launches) outside the capture
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        dc.run_async()
    dc.counts.fill_(-7)
    dc.order.fill_(-7)
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    assert int(dc.counts[0].item()) >= 0
    _check(dc, soa, "graph replay")


def test_async_reports_pending_work():
    # unordered branch logs: the presorted plan fails (-2); finish runs the radix plan
    soa = _lift(20_000, 500, 5, shuffle=True)
    dc = _lib.DeviceCompose(soa)
    dc.run_async()
    dc.torch.cuda.synchronize()
    assert int(dc.counts[0].item()) == -2
    dc.finish()
    _check(dc, soa, "fallback")
    assert dc.last_plan().startswith("radix")
    # moves with a None value: -3 until finish has run their prefix fix-up
    soa = _lift(20_000, 500, 6)
    mv = np.flatnonzero(soa.kind == 0)[::7]
    soa.v0[mv] = -1
    dc = _lib.DeviceCompose(soa)
    dc.run_async()
    dc.torch.cuda.synchronize()
    assert int(dc.counts[0].item()) == -3
    dc.finish()
    _check(dc, soa, "none moves")


def test_long_groups_fail_before_the_tail():
    """>= 4M ops whose timestamp groups (8192 ops) no 2048-op presorted window holds:
    k_khist flags the plan; the synchronous merge launches no tail behind it and takes
    the wide presorted windows, the asynchronous one reports -2 and finish runs them.  Both equal the oracle,
    and so do repeated merges of the same buffers."""
    soa = _lift(4_300_000, 3_000, 19, ops_per_ms=4096, mix=synth.ADVERSARIAL_MIX)
    dc = _lib.DeviceCompose(soa)
    s = dc.torch.cuda.Stream()  # a non-null stream
    for rep in range(3):  # repeated merges of the same buffers
        dc.order.fill_(-7)
        dc.torch.cuda.synchronize()
        dc.run(stream=s)
        _check(dc, soa, f"sync, long groups ({rep})")
        assert dc.last_plan() == "presorted-wide"
    dc.counts.fill_(-7)
    dc.run_async()
    dc.torch.cuda.synchronize()
    assert int(dc.counts[0].item()) == -2
    dc.finish()
    _check(dc, soa, "async, long groups")
    assert dc.last_plan() == "presorted-wide"


def test_async_captured_in_a_graph_forked_tail():
    # >= 4M ops: the table scatter runs on the caller's side stream (event fork/join),
    # so the capture holds both streams
    import torch
    soa = _lift(5_000_000, 100_000, 8)
    dc = _lib.DeviceCompose(soa)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        dc.run_async()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        dc.run_async()
    dc.counts.fill_(-7)
    dc.order.fill_(-7)
    dc.addr.fill_(-7)
    for _ in range(2):
        g.replay()
    torch.cuda.synchronize()
    assert int(dc.counts[0].item()) >= 0
    _check(dc, soa, "graph replay, forked tail")


def test_two_threads_compose_concurrently():
    # smx_compose is reentrant across distinct buffers and streams (include/smx.h):
    # two host threads, each with its own stream, each composing two 5M-op merges
    # (forked table scatter) at the same time on one device
    import threading
    import torch
    soas = [[_lift(5_000_000, 50_000 + 7 * t + k, 20 + 2 * t + k) for k in range(2)] for t in range(2)]
    dcs = [[_lib.DeviceCompose(x) for x in row] for row in soas]
    bar = threading.Barrier(2)
    errors, results = [], {}

    def worker(t):
        try:
            s = torch.cuda.Stream()
            with torch.cuda.stream(s):
                for rep in range(3):
                    for k in range(2):
                        bar.wait()
                        dcs[t][k].run(s)
                s.synchronize()
            for k in range(2):
                results[(t, k)] = dcs[t][k].results()
        except BaseException as e:  # noqa: BLE001 -- reported below
            errors.append(e)
            bar.abort()

    th = [threading.Thread(target=worker, args=(t,)) for t in range(2)]
    for x in th:
        x.start()
    for x in th:
        x.join(timeout=120)
    assert not any(x.is_alive() for x in th), "a compose thread did not finish"
    assert not errors, errors
    for t in range(2):
        for k in range(2):
            ref = oracle.compose(soas[t][k])
            for name, g, r in zip(("order", "addr", "file", "ctx", "conflicts"), results[(t, k)], ref):
                assert np.array_equal(g, r), f"thread {t} merge {k}: {name}"


def test_repeated_merges_read_current_inputs():
    """Repeated smx_compose calls on the same buffers (a non-null stream) recompute from
    the inputs as they are at launch -- new data in the same buffers (same sizes) gives
    that data's composition (nothing is cached between calls; the library's graph replay
    of round 3-5 was removed in round 6)."""
    import torch
    spec = synth.LiftSpec(600_000, 4_000, 31)
    soas = [synth.lift_soa(synth.lift_logs(synth.LiftSpec(**{**spec.__dict__, "seed": sd}))) for sd in (31, 32, 33)]
    assert all(x.n == soas[0].n and x.n_a == soas[0].n_a for x in soas)
    dc = _lib.DeviceCompose(soas[0])
    s = torch.cuda.Stream()
    for rep, soa in enumerate(soas + soas[:1]):
        for name, col, dt in (("kind", soa.kind, np.uint8), ("ts", soa.ts, np.int64), ("hi", soa.oid_hi, np.int64),
                              ("lo", soa.oid_lo, np.int64), ("sym", soa.sym, np.int32), ("v0", soa.v0, np.int32),
                              ("v1", soa.v1, np.int32)):
            getattr(dc, name).copy_(torch.from_numpy(np.ascontiguousarray(col).view(dt)))
        torch.cuda.synchronize()
        dc.run(s)
        s.synchronize()
        _check(dc, soa, f"merge {rep}")


def test_stage_timers_time_every_merge():
    """With the stage timers on every merge's stages get a time, and merges with the
    timers off again still equal the oracle."""
    import torch
    soa = _lift(300_000, 3_000, 34)
    dc = _lib.DeviceCompose(soa)
    s = torch.cuda.Stream()
    L = _lib.lib()
    for _ in range(3):  # untimed merges before the timed ones
        dc.run(s)
    s.synchronize()
    L.smx_set_profiling(1)
    try:
        for rep in range(3):
            L.smx_reset_stage_times()
            dc.run(s)
            s.synchronize()
            st = _lib.stage_times()
            assert st["window"][1] == 1 and st["emit"][1] == 1, st
            assert all(ms > 0 for ms, c in st.values() if c), (rep, st)
    finally:
        L.smx_set_profiling(0)
    _check(dc, soa, "timed merges")
    dc.run(s)
    s.synchronize()
    _check(dc, soa, "untimed merge after the timed merges")

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

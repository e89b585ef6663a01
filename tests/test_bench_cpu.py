"""bench.py's multi-expert roofline aggregation (host logic, no GPU): every expert's probed c5 ops
run on capacity-B buffers with B_e live rows, so an op type's executed and algorithmic work is the
sum over the experts of the capacity-B tally scaled by the expert's routed share B_e / B."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def test_aggregate_expert_ops_scales_by_routed_share():
    import bench
    B = 1024
    per = bench.PROBED["neutron"]["c5"]           # reference FLOPs per image of one c5 pass
    cap_exec = 6.0 * per * B * 4 / 9              # capacity-B executed work of one op (split, sub-pixel)
    raw = {
        "G0.c5.fwd": {"count": 2, "total_ms": 4.0, "exec_flops_per_op": [cap_exec, 0.0, 0.0],
                      "kernel_launches_per_op": 1},
        "G1.c5.fwd": {"count": 2, "total_ms": 2.0, "exec_flops_per_op": [cap_exec, 0.0, 0.0],
                      "kernel_launches_per_op": 1},
    }
    counts = [[768.0, 256.0], [768.0, 256.0]]      # two probe steps, the same routing
    ef = [10.0, 2.0, 1.0]
    stats, live, ef2 = bench.aggregate_expert_ops(raw, counts, ef, "neutron", B)
    assert live == pytest.approx([0.75, 0.25])
    # the step tally is E x one expert's capacity work; live work = sum(live) / E of it
    assert ef2 == pytest.approx([5.0, 1.0, 0.5])
    s = stats["G*.c5.fwd"]
    assert s["count"] == 4 and s["total_ms"] == pytest.approx(6.0) and s["avg_ms"] == pytest.approx(1.5)
    # per op: the mean over the four ops of (share x capacity work)
    assert s["exec_flops_per_op"][0] == pytest.approx(cap_exec * (2 * 0.75 + 2 * 0.25) / 4)
    assert s["alg_per_op"] == pytest.approx(per * B * (2 * 0.75 + 2 * 0.25) / 4)


def test_aggregate_expert_ops_empty_expert():
    """An expert routed no sample contributes its time but no work."""
    import bench
    raw = {"G0.c5.wgrad": {"count": 1, "total_ms": 1.0, "exec_flops_per_op": [8.0, 0.0, 0.0]},
           "G1.c5.wgrad": {"count": 1, "total_ms": 0.5, "exec_flops_per_op": [8.0, 0.0, 0.0]}}
    stats, live, _ = bench.aggregate_expert_ops(raw, [[64.0, 0.0]], [0.0, 0.0, 0.0], "neutron", 64)
    assert live == [1.0, 0.0]
    s = stats["G*.c5.wgrad"]
    assert s["exec_flops_per_op"][0] == pytest.approx(4.0) and s["avg_ms"] == pytest.approx(0.75)

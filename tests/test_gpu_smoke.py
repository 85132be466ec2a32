"""The driver's smoke() checks the flagship operator's output, not only the RHS.

`__graft_entry__.smoke_run` runs 5 CG iterations of the auto-selected
operator (fused5) on the GPU and the same solve with the C++ CPU operator on
the host; smoke() requires them to agree to 1e-10.  A deliberately wrong
table entry of the GPU operator must make that check fail.
"""

import pytest

import __graft_entry__ as entry


@pytest.mark.gpu
def test_smoke_agrees_with_cpu_operator():
    r = entry.smoke_run()
    assert r["op"] == "fused5", r
    assert r["x_max_rel_err"] < 1e-10, r
    entry.smoke()


@pytest.mark.gpu
def test_smoke_fails_on_a_wrong_table():
    r = entry.smoke_run(corrupt_table=True)
    assert r["x_max_rel_err"] > 1e-6, r

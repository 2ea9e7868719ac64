"""Config C5: the synthetic 1 M-triangle random mesh.

The scene is regenerated from its specification (crt_amd/synthetic.py), so
the tree the host build produces must match the reference build's measured
shape (880,933 nodes, 440,467 leaves, 5,723,319 leaf
references, depth 23); the GPU render of a reduced frame must equal the
oracle's bit for bit.
"""
import numpy as np
import pytest

from conftest import bits


@pytest.fixture(scope="module")
def c5():
    from crt_amd.synthetic import c5_scene
    return c5_scene()


def test_c5_tree_shape(c5):
    from crt_amd.native import HostScene
    info = HostScene(c5).info()
    assert info["triangle_count"] == 1_000_000
    assert info["node_count"] == 880_933
    assert info["leaf_count"] == 440_467
    assert info["leaf_ref_count"] == 5_723_319
    assert info["max_depth"] == 23
    assert info["max_leaf_size"] == 16


@pytest.mark.gpu
def test_c5_reduced_frame_bit_exact(c5, oracle):
    from crt_amd import native as N
    from crt_amd.synthetic import c5_scene
    small = c5_scene(width=256, height=144)
    st = N.RendererSettings.default()
    want = oracle.OracleScene(small).render(st)
    gpu = N.HipScene(small)
    got = gpu.render(st)
    assert np.array_equal(bits(got), bits(want))
    wc = N.WorkCounts()
    oracle.OracleScene(small).render(st, counts=wc)
    # the reference-order walk tests exactly the reference's nodes/triangles;
    # the default pruned walk finds the same hits with far fewer tests
    assert N.HipScene(small, traversal=7).count_work(st) == wc.as_dict()
    pruned = gpu.count_work(st)
    assert pruned["hits"] == wc.hits and pruned["traversals"] == wc.traversals
    assert pruned["node_tests"] * 4 < wc.node_tests and pruned["triangle_tests"] * 4 < wc.triangle_tests

"""Host-side shared-prefix group table for the grouped decode-attention kernel (ops.decode_groups)."""
from theroundtaible_amd import ops


def test_groups_basic_and_lone():
    t, nmax = ops.decode_groups(["a", "a", "a", None, "b", "b"], [10, 10, 10, 0, 3, 3], G=4)
    assert t.tolist() == [[0, 3, 10], [0, 3, 10], [0, 3, 10], [3, 1, 0], [4, 2, 3], [4, 2, 3]]
    assert nmax == 3


def test_groups_cut_at_mfma_columns():
    # G=8 (Llama-3-70B): at most 2 sequences per group (16 MFMA columns)
    t, nmax = ops.decode_groups(["a"] * 5, [4] * 5, G=8)
    assert [r[:2] for r in t.tolist()] == [[0, 2], [0, 2], [2, 2], [2, 2], [4, 1]]
    assert t[4].tolist() == [4, 1, 0] and nmax == 2


def test_groups_without_shared_blocks_run_alone():
    t, nmax = ops.decode_groups(["a", "a"], [0, 0], G=4)
    assert t.tolist() == [[0, 1, 0], [1, 1, 0]] and nmax == 1

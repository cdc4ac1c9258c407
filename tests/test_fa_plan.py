"""Prefill attention planning on CPU: when the FA2 kernel pairs each long causal query block with
its short mirror (``ops.fa_pair``; csrc/attention_fa.hip ``pair``)."""
from src import ops


def test_pairing_only_for_small_single_part_grids(monkeypatch):
    monkeypatch.setattr(ops, "FA_PAIR", "auto")
    # one 2K MHA prompt, 4-wave blocks of 128 tokens: 16 blocks x 32 heads = 512 <= 2 x 256 CUs
    assert ops.fa_pair(16, 32, 32, 1)
    # one 8K prompt: 64 blocks x 32 heads = 2048 workgroups, enough to balance by themselves
    assert not ops.fa_pair(64, 32, 32, 1)
    assert not ops.fa_pair(16, 32, 32, 2)  # a context split already shortens the long blocks
    assert not ops.fa_pair(2, 32, 32, 1)   # too few blocks to pair usefully
    monkeypatch.setattr(ops, "FA_PAIR", "1")
    assert ops.fa_pair(64, 32, 32, 1) and not ops.fa_pair(64, 32, 32, 3)
    monkeypatch.setattr(ops, "FA_PAIR", "0")
    assert not ops.fa_pair(16, 32, 32, 1)

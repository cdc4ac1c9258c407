"""Prefill attention planning on CPU: when the FA2 kernel pairs each long causal query block with
its short mirror (``ops.fa_pair``; csrc/attention_fa.hip ``pair``)."""
from src import ops


def test_pairing_whenever_the_context_is_not_split(monkeypatch):
    monkeypatch.setattr(ops, "FA_PAIR", "auto")
    assert ops.fa_pair(16, 32, 32, 1)      # one 2K MHA prompt, 4-wave blocks of 128 tokens
    assert ops.fa_pair(64, 32, 8, 1)       # 64 short prompts: two blocks per workgroup
    assert not ops.fa_pair(16, 32, 32, 2)  # a context split already shortens the long blocks
    assert not ops.fa_pair(1, 32, 32, 1)   # nothing to pair
    monkeypatch.setattr(ops, "FA_PAIR", "1")
    assert ops.fa_pair(64, 32, 32, 1) and not ops.fa_pair(64, 32, 32, 3)
    monkeypatch.setattr(ops, "FA_PAIR", "0")
    assert not ops.fa_pair(16, 32, 32, 1)

"""Model configurations.

The reference resolves ``--model`` through ``AutoModelForCausalLM.from_pretrained``
(reference src/llama_partition.py:495) and accepts only ``model_type`` in
{llama, mistral, mixtral} (src/llama_partition.py:81-83).  Here a model name
resolves to, in order:

1. a local directory holding a Hugging Face ``config.json`` (weights are then read
   from its safetensors shards, see ``models.weights``);
2. a built-in preset for the configurations named in BASELINE.json / SURVEY.md
   (Llama-2-7B, Llama-3(.1)-8B, Llama-3-70B, GPT-2) plus tiny test models.

The GPU box has no network, so presets are used with synthetic random-init weights.
"""
from __future__ import annotations

import dataclasses
import json
import os
from typing import Optional

SUPPORTED_TYPES = ("llama", "mistral", "mixtral", "gpt2")


@dataclasses.dataclass
class ModelConfig:
    model_type: str = "llama"
    vocab_size: int = 32000
    hidden_size: int = 4096
    intermediate_size: int = 11008
    num_hidden_layers: int = 32
    num_attention_heads: int = 32
    num_key_value_heads: int = 32
    head_dim: int = 128
    rms_norm_eps: float = 1e-5
    layer_norm_eps: float = 1e-5
    rope_theta: float = 10000.0
    rope_scaling: Optional[dict] = None
    max_position_embeddings: int = 4096
    tie_word_embeddings: bool = False
    bos_token_id: int = 1
    eos_token_id: int = 2
    name: str = "custom"
    # Mixtral sparse MoE MLP (HF MixtralSparseMoeBlock): E experts, top-k softmax routing
    num_local_experts: int = 0
    num_experts_per_tok: int = 2
    # Mistral / Mixtral sliding-window attention (None = full causal attention)
    sliding_window: Optional[int] = None

    @property
    def is_moe(self) -> bool:
        return self.num_local_experts > 0

    @property
    def kv_dim(self) -> int:
        return self.num_key_value_heads * self.head_dim

    @property
    def q_dim(self) -> int:
        return self.num_attention_heads * self.head_dim

    @property
    def n_rep(self) -> int:
        return self.num_attention_heads // self.num_key_value_heads

    def layer_param_bytes(self, bytes_per_param: float = 2.0) -> int:
        """Weights of one decoder block (survey V11 `get_block_size`)."""
        H, F = self.hidden_size, self.intermediate_size
        if self.model_type == "gpt2":
            n = 4 * H * H + 2 * H * F + 9 * H + F
        else:
            mlp = self.num_local_experts * (3 * H * F + H) if self.is_moe else 3 * H * F
            n = H * (self.q_dim + 2 * self.kv_dim) + self.q_dim * H + mlp + 2 * H
        return int(n * bytes_per_param)

    def kv_bytes_per_token_per_layer(self, bytes_per_elt: int = 2) -> int:
        return 2 * self.kv_dim * bytes_per_elt

    def validate(self) -> None:
        if self.model_type not in SUPPORTED_TYPES:
            raise ValueError(f"unsupported model_type {self.model_type!r}; supported: {SUPPORTED_TYPES}")
        if self.num_attention_heads % self.num_key_value_heads:
            raise ValueError("num_attention_heads must be a multiple of num_key_value_heads")
        if self.head_dim % 8:
            raise ValueError("head_dim must be a multiple of 8")
        if self.is_moe and not (1 <= self.num_experts_per_tok <= self.num_local_experts <= 64):
            raise ValueError("MoE needs 1 <= num_experts_per_tok <= num_local_experts <= 64")

    def to_dict(self) -> dict:
        return dataclasses.asdict(self)

    @classmethod
    def from_hf_dict(cls, d: dict, name: str = "custom") -> "ModelConfig":
        mt = d.get("model_type", "llama")
        if mt == "gpt2":
            H = d.get("n_embd", d.get("hidden_size", 768))
            nh = d.get("n_head", d.get("num_attention_heads", 12))
            return cls(model_type="gpt2", vocab_size=d.get("vocab_size", 50257), hidden_size=H,
                       intermediate_size=d.get("n_inner") or 4 * H, num_hidden_layers=d.get("n_layer", 12),
                       num_attention_heads=nh, num_key_value_heads=nh, head_dim=H // nh,
                       layer_norm_eps=d.get("layer_norm_epsilon", 1e-5),
                       max_position_embeddings=d.get("n_positions", 1024), tie_word_embeddings=True,
                       bos_token_id=d.get("bos_token_id", 50256), eos_token_id=d.get("eos_token_id", 50256),
                       name=name)
        H = d["hidden_size"]
        nh = d["num_attention_heads"]
        eos = d.get("eos_token_id", 2)
        if isinstance(eos, list):
            eos = eos[0]
        # transformers >= 5 nests rope settings under ``rope_parameters``
        rp = d.get("rope_parameters") or {}
        theta = d.get("rope_theta") or rp.get("rope_theta", 10000.0)
        scaling = d.get("rope_scaling") or (rp if rp.get("rope_type", "default") != "default" else None)
        return cls(model_type=mt, vocab_size=d["vocab_size"], hidden_size=H,
                   intermediate_size=d["intermediate_size"], num_hidden_layers=d["num_hidden_layers"],
                   num_attention_heads=nh, num_key_value_heads=d.get("num_key_value_heads", nh),
                   head_dim=d.get("head_dim") or H // nh, rms_norm_eps=d.get("rms_norm_eps", 1e-5),
                   rope_theta=theta, rope_scaling=scaling,
                   max_position_embeddings=d.get("max_position_embeddings", 4096),
                   tie_word_embeddings=d.get("tie_word_embeddings", False),
                   bos_token_id=d.get("bos_token_id", 1) or 1, eos_token_id=eos, name=name,
                   num_local_experts=int(d.get("num_local_experts", 0) or 0) if mt == "mixtral" else 0,
                   num_experts_per_tok=int(d.get("num_experts_per_tok", 2) or 2),
                   sliding_window=d.get("sliding_window"))


PRESETS = {
    "llama2-7b": ModelConfig(name="llama2-7b"),
    "llama3-8b": ModelConfig(vocab_size=128256, intermediate_size=14336, num_key_value_heads=8,
                             rope_theta=500000.0, max_position_embeddings=8192, bos_token_id=128000,
                             eos_token_id=128001, name="llama3-8b"),
    "llama3-70b": ModelConfig(vocab_size=128256, hidden_size=8192, intermediate_size=28672, num_hidden_layers=80,
                              num_attention_heads=64, num_key_value_heads=8, rope_theta=500000.0,
                              max_position_embeddings=8192, bos_token_id=128000, eos_token_id=128001,
                              name="llama3-70b"),
    "gpt2": ModelConfig(model_type="gpt2", vocab_size=50257, hidden_size=768, intermediate_size=3072,
                        num_hidden_layers=12, num_attention_heads=12, num_key_value_heads=12, head_dim=64,
                        max_position_embeddings=1024, tie_word_embeddings=True, bos_token_id=50256,
                        eos_token_id=50256, name="gpt2"),
    "mistral-7b": ModelConfig(model_type="mistral", intermediate_size=14336, num_key_value_heads=8,
                              max_position_embeddings=32768, sliding_window=4096, name="mistral-7b"),
    "mixtral-8x7b": ModelConfig(model_type="mixtral", intermediate_size=14336, num_key_value_heads=8,
                                rope_theta=1e6, max_position_embeddings=32768, num_local_experts=8,
                                num_experts_per_tok=2, name="mixtral-8x7b"),
    # small models for tests / CPU plumbing
    "tiny-mixtral": ModelConfig(model_type="mixtral", vocab_size=512, hidden_size=256, intermediate_size=256,
                                num_hidden_layers=4, num_attention_heads=4, num_key_value_heads=2, head_dim=64,
                                max_position_embeddings=1024, num_local_experts=4, num_experts_per_tok=2,
                                name="tiny-mixtral"),
    "tiny-llama": ModelConfig(vocab_size=512, hidden_size=256, intermediate_size=512, num_hidden_layers=4,
                              num_attention_heads=4, num_key_value_heads=2, head_dim=64,
                              max_position_embeddings=1024, name="tiny-llama"),
    "small-llama": ModelConfig(vocab_size=1024, hidden_size=512, intermediate_size=1024, num_hidden_layers=8,
                               num_attention_heads=4, num_key_value_heads=4, head_dim=128,
                               max_position_embeddings=2048, name="small-llama"),
    "tiny-gpt2": ModelConfig(model_type="gpt2", vocab_size=512, hidden_size=128, intermediate_size=512,
                             num_hidden_layers=4, num_attention_heads=2, num_key_value_heads=2, head_dim=64,
                             max_position_embeddings=512, tie_word_embeddings=True, bos_token_id=0,
                             eos_token_id=511, name="tiny-gpt2"),
}

_ALIASES = {
    "llama-2-7b": "llama2-7b",
    "llama2-7b": "llama2-7b",
    "llama-3.1-8b": "llama3-8b",
    "llama-3-8b": "llama3-8b",
    "llama3-8b": "llama3-8b",
    "llama3.1-8b": "llama3-8b",
    "llama-3-70b": "llama3-70b",
    "llama-3.1-70b": "llama3-70b",
    "llama3-70b": "llama3-70b",
    "mixtral-8x7b": "mixtral-8x7b",
    "mistral-7b": "mistral-7b",
}


def resolve_model(name: str) -> ModelConfig:
    """Resolve ``--model`` to a config (local HF dir first, then presets)."""
    if os.path.isdir(name) and os.path.exists(os.path.join(name, "config.json")):
        with open(os.path.join(name, "config.json")) as f:
            cfg = ModelConfig.from_hf_dict(json.load(f), name=name)
        cfg.validate()
        return cfg
    key = name.lower().rstrip("/")
    if key in PRESETS:
        return dataclasses.replace(PRESETS[key])
    base = key.split("/")[-1]
    base = base.replace("meta-", "").replace("-hf", "").replace("-chat", "").replace("-instruct", "")
    if base in PRESETS:
        return dataclasses.replace(PRESETS[base])
    for alias, preset in _ALIASES.items():
        if alias in base:
            return dataclasses.replace(PRESETS[preset], name=name)
    if base.startswith("gpt2"):
        return dataclasses.replace(PRESETS["gpt2"], name=name)
    raise ValueError(f"unknown model {name!r}: pass a local HF directory or one of {sorted(PRESETS)}")

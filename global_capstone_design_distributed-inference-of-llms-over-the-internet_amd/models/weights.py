"""Per-stage weights: synthetic random init or HF checkpoint loading of ONLY the stage's keys.

The reference loads the whole HF model on CPU in every stage process and then prunes
``model.layers`` (reference src/llama_partition.py:495-530); the vendored Petals server
instead reads only ``model.layers.{i}.*`` from the sharded checkpoint
(reference petals/server/from_pretrained.py:35-128).  Here a stage reads only its own
blocks (plus embeddings / final norm / lm_head when its role needs them) straight from
the safetensors shards, and lays them out for the MI355X kernels:

* q/k/v fused into one ``qkv`` matrix [(nh + 2 nkv) * D, H] -> one GEMM per layer;
* gate/up fused into ``gate_up`` [2F, H] with rows interleaved in 16-row blocks
  ([g0..g15, u0..u15, g16..g31, ...]) so the GEMM epilogue can apply SwiGLU in registers;
* everything resident on the GPU (no per-forward CPU<->GPU streaming, unlike
  src/llama_partition.py:169-180, :233-293 of the reference).

Random init is deterministic per (seed, block index): a model split into any number of
stages gets bit-identical weights, which the pipeline-equivalence tests rely on.
"""
from __future__ import annotations

import dataclasses
import glob
import json
import os
from typing import Dict, List, Optional

import torch

from .config import ModelConfig
from ..ops.reference import GU_BLOCK

INIT_STD = 0.02


def interleave_gate_up(gate: torch.Tensor, up: torch.Tensor) -> torch.Tensor:
    F, H = gate.shape
    assert F % GU_BLOCK == 0, "intermediate_size must be a multiple of 16"
    return torch.stack([gate.view(F // GU_BLOCK, GU_BLOCK, H), up.view(F // GU_BLOCK, GU_BLOCK, H)], 1).reshape(2 * F, H)


def split_gate_up(gu: torch.Tensor):
    F2, H = gu.shape
    v = gu.view(F2 // (2 * GU_BLOCK), 2, GU_BLOCK, H)
    return v[:, 0].reshape(F2 // 2, H), v[:, 1].reshape(F2 // 2, H)


@dataclasses.dataclass
class LlamaLayer:
    input_norm: torch.Tensor
    qkv: torch.Tensor
    o: torch.Tensor
    post_norm: torch.Tensor
    gate_up: torch.Tensor
    down: torch.Tensor
    # fragment-native packed copies for the decode GEMM (ops.pack_weight); None until packed
    qkv_p: Optional[torch.Tensor] = None
    o_p: Optional[torch.Tensor] = None
    gate_up_p: Optional[torch.Tensor] = None
    down_p: Optional[torch.Tensor] = None
    # fp8 e4m3 W8A8 copies (ops.pack_weight_fp8): packed uint8 + per-output-channel fp32 scale
    qkv_q: Optional[torch.Tensor] = None
    qkv_s: Optional[torch.Tensor] = None
    o_q: Optional[torch.Tensor] = None
    o_s: Optional[torch.Tensor] = None
    gate_up_q: Optional[torch.Tensor] = None
    gate_up_s: Optional[torch.Tensor] = None
    down_q: Optional[torch.Tensor] = None
    down_s: Optional[torch.Tensor] = None
    # fp8 W8A16 copies (ops.w8_from_fp8: the bf16 fragment order at 1 byte per weight) + fp32
    # per-output-channel scales, for the fused-norm decode GEMMs of an fp8 stage
    qkv_w8: Optional[torch.Tensor] = None
    qkv_ws: Optional[torch.Tensor] = None
    o_w8: Optional[torch.Tensor] = None
    o_ws: Optional[torch.Tensor] = None
    gate_up_w8: Optional[torch.Tensor] = None
    gate_up_ws: Optional[torch.Tensor] = None
    down_w8: Optional[torch.Tensor] = None
    down_ws: Optional[torch.Tensor] = None
    # Mixtral sparse-MoE block (HF MixtralSparseMoeBlock): ``router`` [E, H]; gate_up / down
    # (and their packed copies) are then stacked per expert: [E, 2F, H] / [E, H, F]
    router: Optional[torch.Tensor] = None
    router_p: Optional[torch.Tensor] = None  # router padded to 16 rows, packed (decode GEMM)
    folded: bool = False  # qkv_p / gate_up_p carry the input / post-attention norm weights

    PROJ = ("qkv", "o", "gate_up", "down")

    @property
    def moe(self) -> bool:
        return self.router is not None

    @property
    def fp8(self) -> bool:
        return self.qkv_q is not None or self.qkv_w8 is not None

    @property
    def w8(self) -> bool:
        return self.qkv_w8 is not None

    def dense(self, name: str, dtype=torch.bfloat16) -> torch.Tensor:
        """Row-major weight ``name`` (dequantized on the fly when only an fp8 copy is kept; a
        W8A16 layer's qkv / gate_up then carry the folded norm weights, see ``folded``)."""
        w = getattr(self, name)
        if w is not None:
            return w
        from .. import ops

        if getattr(self, name + "_w8") is not None:
            return ops.unpack_weight_w8(getattr(self, name + "_w8"), getattr(self, name + "_ws"), dtype)
        return ops.unpack_weight_fp8(getattr(self, name + "_q"), getattr(self, name + "_s"), dtype)


@dataclasses.dataclass
class GPT2Layer:
    ln1_w: torch.Tensor
    ln1_b: torch.Tensor
    attn_w: torch.Tensor  # [3H, H] (HF Conv1D weight transposed)
    attn_b: torch.Tensor
    proj_w: torch.Tensor
    proj_b: torch.Tensor
    ln2_w: torch.Tensor
    ln2_b: torch.Tensor
    fc_w: torch.Tensor
    fc_b: torch.Tensor
    fc2_w: torch.Tensor
    fc2_b: torch.Tensor


@dataclasses.dataclass
class StageWeights:
    cfg: ModelConfig
    start: int
    end: int
    layers: list
    embed: Optional[torch.Tensor] = None        # [V, H] (gpt2: wte)
    pos_embed: Optional[torch.Tensor] = None    # gpt2 wpe [P, H]
    final_norm: Optional[torch.Tensor] = None   # llama [H]; gpt2 ln_f weight
    final_norm_b: Optional[torch.Tensor] = None  # gpt2 ln_f bias
    lm_head: Optional[torch.Tensor] = None      # [V, H]
    lm_head_p: Optional[torch.Tensor] = None    # packed lm_head (V padded to a multiple of 16)
    lm_head_folded: bool = False                # lm_head_p carries final_norm in its K columns

    @property
    def has_embed(self) -> bool:
        return self.embed is not None

    @property
    def has_head(self) -> bool:
        return self.lm_head is not None

    def nbytes(self) -> int:
        n = 0
        for t in self.tensors():
            n += t.numel() * t.element_size()
        return n

    def pack_for_decode(self, fold_norms: bool = False) -> None:
        """Add fragment-native copies of every projection (MI355X decode GEMM layout).

        The row-major weights stay for the hipBLASLt prefill path: 2x weight bytes, which
        288 GB of HBM affords (13.5 GB -> 27 GB for Llama-2-7B on one GPU).

        ``fold_norms``: the packed qkv / gate_up copies carry the RMSNorm weight folded into
        their K columns (W' = W diag(g)) for the fused-norm decode path, whose GEMMs take the raw
        residual stream and apply rsqrt(mean x^2) per row in the epilogue (ops/csrc/gemm.hip).
        """
        from .. import ops

        for lay in self.layers:
            if isinstance(lay, LlamaLayer) and lay.qkv_p is None and lay.qkv is not None:
                if fold_norms and not lay.moe:
                    lay.qkv_p = ops.pack_weight((lay.qkv.float() * lay.input_norm.float()[None, :])
                                                .to(lay.qkv.dtype).contiguous())
                    lay.o_p = ops.pack_weight(lay.o)
                    lay.gate_up_p = ops.pack_weight((lay.gate_up.float() * lay.post_norm.float()[None, :])
                                                    .to(lay.gate_up.dtype).contiguous())
                    lay.down_p = ops.pack_weight(lay.down)
                    lay.folded = True
                    continue
                lay.qkv_p = ops.pack_weight(lay.qkv)
                lay.o_p = ops.pack_weight(lay.o)
                if lay.moe:
                    lay.gate_up_p = torch.stack([ops.pack_weight(w) for w in lay.gate_up])
                    lay.down_p = torch.stack([ops.pack_weight(w) for w in lay.down])
                    E, H = lay.router.shape
                    lay.router_p = ops.pack_weight(torch.cat([lay.router, lay.router.new_zeros((-E) % 16, H)]))
                else:
                    lay.gate_up_p = ops.pack_weight(lay.gate_up)
                    lay.down_p = ops.pack_weight(lay.down)
        if self.lm_head is not None and self.lm_head_p is None and self.cfg.model_type != "gpt2":
            V, H = self.lm_head.shape
            if H % 32 == 0:
                pad = (-V) % 16
                w = self.lm_head if pad == 0 else torch.cat([self.lm_head, self.lm_head.new_zeros(pad, H)])
                # fused-norm decode: the final RMSNorm weight folded in as for qkv / gate_up, so a
                # decode step's lm_head reads the packed residual stream + its row statistics
                # (no final norm launch); other steps normalise with a unit weight first
                fold = fold_norms and self.final_norm is not None
                if fold:
                    w = (w.float() * self.final_norm.float()[None, :]).to(w.dtype)
                self.lm_head_p = ops.pack_weight(w.contiguous())
                self.lm_head_folded = fold

    def quantize_fp8(self, drop_dense: bool = True) -> None:
        """fp8 (OCP e4m3) W8A8 weights for every projection (the 70B fp8 MFMA path).

        ``drop_dense`` frees the bf16 copies (the prefill path then dequantizes one layer at a
        time), halving resident weight bytes: Llama-3-70B fits ONE MI355X (~70 GB) with room
        for a large KV cache.  Embeddings, norms and lm_head stay bf16.
        """
        from .. import ops

        if self.cfg.is_moe:
            raise ValueError("fp8 W8A8 weights are not supported for MoE (Mixtral) models")
        for lay in self.layers:
            if not isinstance(lay, LlamaLayer) or lay.fp8:
                continue
            for name in LlamaLayer.PROJ:
                q, sc = ops.pack_weight_fp8(getattr(lay, name))
                setattr(lay, name + "_q", q)
                setattr(lay, name + "_s", sc)
                if drop_dense:
                    setattr(lay, name, None)
                    setattr(lay, name + "_p", None)

    def prepare_w8a16(self, fold_norms: bool = True) -> None:
        """Convert every fp8 layer to the W8A16 layout (ops.w8_from_fp8) and drop the W8A8
        copies.  ``fold_norms``: qkv / gate_up are dequantized, multiplied by the input /
        post-attention RMSNorm weight along K and re-quantized (W' = W diag(g), per-output-channel
        scales), as the bf16 fused-norm path folds them into its packed weights; ``folded`` is set
        and every path over these weights normalises with a unit RMSNorm weight."""
        from .. import ops

        for lay in self.layers:
            if not isinstance(lay, LlamaLayer) or lay.w8 or lay.qkv_q is None:
                continue
            for name, g in (("qkv", lay.input_norm), ("o", None), ("gate_up", lay.post_norm), ("down", None)):
                q, sc = getattr(lay, name + "_q"), getattr(lay, name + "_s")
                if fold_norms and g is not None:
                    w = ops.unpack_weight_fp8(q, sc, torch.float32) * g.float()[None, :]
                    q, sc = ops.pack_weight_fp8(w)
                    del w
                setattr(lay, name + "_w8", ops.w8_from_fp8(q))
                setattr(lay, name + "_ws", sc)
                setattr(lay, name + "_q", None)
                setattr(lay, name + "_s", None)
            lay.folded = bool(fold_norms)

    @property
    def fp8(self) -> bool:
        return bool(self.layers) and all(isinstance(L, LlamaLayer) and L.fp8 for L in self.layers)

    @property
    def w8(self) -> bool:
        return bool(self.layers) and all(isinstance(L, LlamaLayer) and L.w8 for L in self.layers)

    def tensors(self):
        seen = set()
        for lay in self.layers:
            for f in dataclasses.fields(lay):
                t = getattr(lay, f.name)
                if t is not None and id(t) not in seen:
                    seen.add(id(t))
                    yield t
        for t in (self.embed, self.pos_embed, self.final_norm, self.final_norm_b, self.lm_head, self.lm_head_p):
            if t is not None and id(t) not in seen:
                seen.add(id(t))
                yield t


def _gen(device, seed: int):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return g


def _randn(shape, g, device, dtype, std=INIT_STD):
    t = torch.empty(shape, dtype=torch.float32, device=device)
    t.normal_(0.0, std, generator=g)
    return t.to(dtype)


def _random_llama_layer(cfg: ModelConfig, idx: int, device, dtype, seed: int) -> LlamaLayer:
    g = _gen(device, seed * 100003 + idx + 1)
    H, F = cfg.hidden_size, cfg.intermediate_size
    qkv = _randn((cfg.q_dim + 2 * cfg.kv_dim, H), g, device, dtype)
    o = _randn((H, cfg.q_dim), g, device, dtype)
    ones = torch.ones(H, dtype=dtype, device=device)
    if cfg.is_moe:
        E = cfg.num_local_experts
        router = _randn((E, H), g, device, dtype)
        gu = torch.empty((E, 2 * F, H), dtype=dtype, device=device)
        dn = torch.empty((E, H, F), dtype=dtype, device=device)
        for e in range(E):
            gu[e] = interleave_gate_up(_randn((F, H), g, device, dtype), _randn((F, H), g, device, dtype))
            dn[e] = _randn((H, F), g, device, dtype)
        return LlamaLayer(ones, qkv, o, ones.clone(), gu, dn, router=router)
    gate = _randn((F, H), g, device, dtype)
    up = _randn((F, H), g, device, dtype)
    down = _randn((H, F), g, device, dtype)
    return LlamaLayer(ones, qkv, o, ones.clone(), interleave_gate_up(gate, up), down)


def _random_gpt2_layer(cfg: ModelConfig, idx: int, device, dtype, seed: int) -> GPT2Layer:
    g = _gen(device, seed * 100003 + idx + 1)
    H, F = cfg.hidden_size, cfg.intermediate_size
    z = lambda n: torch.zeros(n, dtype=dtype, device=device)  # noqa: E731
    o = lambda n: torch.ones(n, dtype=dtype, device=device)  # noqa: E731
    return GPT2Layer(o(H), z(H), _randn((3 * H, H), g, device, dtype), z(3 * H), _randn((H, H), g, device, dtype),
                     z(H), o(H), z(H), _randn((F, H), g, device, dtype), z(F), _randn((H, F), g, device, dtype), z(H))


def random_stage_weights(cfg: ModelConfig, start: int, end: int, *, has_embed: bool, has_head: bool, device,
                         dtype=torch.bfloat16, seed: int = 0, fp8: bool = False) -> StageWeights:
    """``fp8``: quantize each block as soon as it is generated (bf16 copies dropped), so a
    70B stage never holds its full bf16 weights."""
    device = torch.device(device)
    mk = _random_gpt2_layer if cfg.model_type == "gpt2" else _random_llama_layer
    layers = []
    for i in range(start, end):
        lay = mk(cfg, i, device, dtype, seed)
        if fp8 and isinstance(lay, LlamaLayer):
            one = StageWeights(cfg, i, i + 1, [lay])
            one.quantize_fp8(drop_dense=True)
        layers.append(lay)
    sw = StageWeights(cfg, start, end, layers)
    H, V = cfg.hidden_size, cfg.vocab_size
    if has_embed or (has_head and cfg.tie_word_embeddings):
        g = _gen(device, seed * 100003 + 7919)
        emb = _randn((V, H), g, device, dtype)
        if has_embed:
            sw.embed = emb
        if cfg.model_type == "gpt2" and has_embed:
            sw.pos_embed = _randn((cfg.max_position_embeddings, H), _gen(device, seed * 100003 + 7927), device,
                                  dtype, std=0.01)
        if has_head and cfg.tie_word_embeddings:
            sw.lm_head = emb
    if has_head:
        sw.final_norm = torch.ones(H, dtype=dtype, device=device)
        if cfg.model_type == "gpt2":
            sw.final_norm_b = torch.zeros(H, dtype=dtype, device=device)
        if sw.lm_head is None:
            sw.lm_head = _randn((V, H), _gen(device, seed * 100003 + 7937), device, dtype)
    return sw


# ------------------------------------------------------------------ checkpoint loading
SAFE_INDEX = "model.safetensors.index.json"
BIN_INDEX = "pytorch_model.bin.index.json"


def checkpoint_files(path: str) -> Optional[str]:
    """Which weight format a local HF directory holds: "safetensors", "bin" or None.

    Same lookup order as upstream Petals ``INDEX_FILES`` / ``_find_index_file``
    (reference petals/server/from_pretrained.py:131-159): sharded safetensors, sharded
    ``.bin``, then single-file variants."""
    if os.path.exists(os.path.join(path, SAFE_INDEX)) or glob.glob(os.path.join(path, "*.safetensors")):
        return "safetensors"
    if os.path.exists(os.path.join(path, BIN_INDEX)) or glob.glob(os.path.join(path, "*.bin")):
        return "bin"
    return None


class _Checkpoint:
    """Key -> shard lookup over a local HF directory (sharded or single-file; safetensors or
    ``pytorch_model*.bin``).

    ``.bin`` shards are read with ``torch.load(weights_only=True, mmap=True)``: the restricted
    unpickler executes nothing from the file, and the memory map means only the tensors a stage
    actually asks for are paged in (upstream ``_load_state_dict_from_local_file``,
    petals/server/from_pretrained.py:216-224, loads whole shards)."""

    def __init__(self, path: str):
        self.path = path
        self._handles: Dict[str, object] = {}
        self.kind = checkpoint_files(path)
        if self.kind is None:
            raise FileNotFoundError(f"no safetensors or pytorch_model*.bin weights under {path}")
        self.key_to_file: Dict[str, str] = {}
        index = os.path.join(path, SAFE_INDEX if self.kind == "safetensors" else BIN_INDEX)
        if os.path.exists(index):
            with open(index) as f:
                wm = json.load(f)["weight_map"]
            self.key_to_file = {k: os.path.join(path, v) for k, v in wm.items()}
        else:
            pattern = "*.safetensors" if self.kind == "safetensors" else "*.bin"
            for fn in sorted(glob.glob(os.path.join(path, pattern))):
                for k in self._open(fn).keys():
                    self.key_to_file[k] = fn

    def _open(self, fn: str):
        h = self._handles.get(fn)
        if h is not None:
            return h
        if self.kind == "safetensors":
            from safetensors import safe_open

            h = safe_open(fn, framework="pt")
        else:
            try:
                h = torch.load(fn, map_location="cpu", weights_only=True, mmap=True)
            except RuntimeError:  # legacy (non-zip) serialization cannot be memory-mapped
                h = torch.load(fn, map_location="cpu", weights_only=True)
            if not isinstance(h, dict):
                raise ValueError(f"{fn}: expected a state dict, got {type(h).__name__}")
        self._handles[fn] = h
        return h

    def has(self, key: str) -> bool:
        return key in self.key_to_file

    def get(self, key: str) -> torch.Tensor:
        h = self._open(self.key_to_file[key])
        return h.get_tensor(key) if self.kind == "safetensors" else h[key]


def load_stage_weights(cfg: ModelConfig, path: str, start: int, end: int, *, has_embed: bool, has_head: bool,
                       device, dtype=torch.bfloat16) -> StageWeights:
    ck = _Checkpoint(path)
    dev = torch.device(device)

    def t(key):
        return ck.get(key).to(device=dev, dtype=dtype)

    layers: List = []
    if cfg.model_type == "gpt2":
        pre = "transformer." if ck.has("transformer.wte.weight") else ""
        for i in range(start, end):
            p = f"{pre}h.{i}."
            layers.append(GPT2Layer(t(p + "ln_1.weight"), t(p + "ln_1.bias"), t(p + "attn.c_attn.weight").t().contiguous(),
                                    t(p + "attn.c_attn.bias"), t(p + "attn.c_proj.weight").t().contiguous(),
                                    t(p + "attn.c_proj.bias"), t(p + "ln_2.weight"), t(p + "ln_2.bias"),
                                    t(p + "mlp.c_fc.weight").t().contiguous(), t(p + "mlp.c_fc.bias"),
                                    t(p + "mlp.c_proj.weight").t().contiguous(), t(p + "mlp.c_proj.bias")))
        sw = StageWeights(cfg, start, end, layers)
        if has_embed:
            sw.embed = t(pre + "wte.weight")
            sw.pos_embed = t(pre + "wpe.weight")
        if has_head:
            sw.final_norm, sw.final_norm_b = t(pre + "ln_f.weight"), t(pre + "ln_f.bias")
            sw.lm_head = sw.embed if sw.embed is not None else t(pre + "wte.weight")
        return sw
    for i in range(start, end):
        p = f"model.layers.{i}."
        qkv = torch.cat([t(p + "self_attn.q_proj.weight"), t(p + "self_attn.k_proj.weight"),
                         t(p + "self_attn.v_proj.weight")], 0).contiguous()
        if cfg.is_moe:  # HF MixtralSparseMoeBlock: gate = router, experts.j.{w1 gate, w3 up, w2 down}
            m = p + "block_sparse_moe."
            E = cfg.num_local_experts
            gu = torch.stack([interleave_gate_up(t(f"{m}experts.{j}.w1.weight"), t(f"{m}experts.{j}.w3.weight"))
                              for j in range(E)])
            dn = torch.stack([t(f"{m}experts.{j}.w2.weight") for j in range(E)])
            layers.append(LlamaLayer(t(p + "input_layernorm.weight"), qkv, t(p + "self_attn.o_proj.weight"),
                                     t(p + "post_attention_layernorm.weight"), gu, dn, router=t(m + "gate.weight")))
            continue
        gu = interleave_gate_up(t(p + "mlp.gate_proj.weight"), t(p + "mlp.up_proj.weight")).contiguous()
        layers.append(LlamaLayer(t(p + "input_layernorm.weight"), qkv, t(p + "self_attn.o_proj.weight"),
                                 t(p + "post_attention_layernorm.weight"), gu, t(p + "mlp.down_proj.weight")))
    sw = StageWeights(cfg, start, end, layers)
    if has_embed:
        sw.embed = t("model.embed_tokens.weight")
    if has_head:
        sw.final_norm = t("model.norm.weight")
        if ck.has("lm_head.weight"):
            sw.lm_head = t("lm_head.weight")
        else:  # tied embeddings
            sw.lm_head = sw.embed if sw.embed is not None else t("model.embed_tokens.weight")
    return sw


def build_stage_weights(cfg: ModelConfig, model: str, start: int, end: int, *, has_embed: bool, has_head: bool,
                        device, dtype=torch.bfloat16, seed: int = 0) -> StageWeights:
    """Checkpoint weights when ``model`` is a local HF directory, synthetic weights for presets.

    A directory without loadable weights is an error: silently serving a real config with
    random weights would produce garbage that looks like a working server."""
    if os.path.isdir(model):
        if checkpoint_files(model) is None:
            raise FileNotFoundError(f"--model {model!r} is a directory without *.safetensors or pytorch_model*.bin "
                                    f"weights (pass a preset name such as llama2-7b for synthetic weights)")
        return load_stage_weights(cfg, model, start, end, has_embed=has_embed, has_head=has_head, device=device,
                                  dtype=dtype)
    return random_stage_weights(cfg, start, end, has_embed=has_embed, has_head=has_head, device=device, dtype=dtype,
                                seed=seed)

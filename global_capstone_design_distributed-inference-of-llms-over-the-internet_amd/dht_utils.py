"""Registry record schema for the swarm (same keys and fields as the reference).

Record families (reference src/dht_utils.py:20-281, src/main.py:517-526, :656-666):

=======================================  ===========  =============================================
key                                      subkey       value
=======================================  ===========  =============================================
``mini_petals:stage{N}``                 peer id      peer_id, timestamp, stage, p2p_maddrs (+ blocks,
                                                      throughput in load-balancing mode)
``petals:server:{model}:{peer_id}``      -            peer_id, timestamp, start_block, end_block,
                                                      throughput, state, server_address, p2p_maddrs,
                                                      final_stage
``petals:module:{model}:block_{i}``      peer id      peer_id, timestamp, block_idx, start_block,
                                                      end_block, throughput, state, p2p_maddrs,
                                                      final_stage
=======================================  ===========  =============================================
"""
from __future__ import annotations

import logging
from typing import Any, Dict, List, Optional

from .comm.registry import DHT, get_dht_time
from .load_balancing import RemoteModuleInfo, ServerInfo, ServerState

logger = logging.getLogger(__name__)

MODULE_KEY_PREFIX = "petals:module:"
SERVER_KEY_PREFIX = "petals:server:"
STAGE_KEY_PREFIX = "mini_petals:stage"
DEFAULT_TTL = 45.0


def get_stage_key(stage: int) -> str:
    return f"{STAGE_KEY_PREFIX}{stage}"


def get_module_key(block_idx: int, model_name: str = "default") -> str:
    return f"{MODULE_KEY_PREFIX}{model_name}:block_{block_idx}"


def get_server_key(peer_id, model_name: str = "default") -> str:
    return f"{SERVER_KEY_PREFIX}{model_name}:{peer_id}"


def register_stage_on_dht(dht: DHT, stage: int, peer_id, p2p_maddrs: List[str], ttl: float = DEFAULT_TTL,
                          **extra) -> bool:
    rec = {"peer_id": str(peer_id), "timestamp": get_dht_time(), "stage": int(stage), "p2p_maddrs": list(p2p_maddrs)}
    rec.update(extra)
    return dht.store(get_stage_key(stage), rec, get_dht_time() + ttl, subkey=str(peer_id))


def register_server_on_dht(dht: DHT, peer_id, start_block: int, end_block: int, throughput: float,
                           model_name: str = "default", server_address: Optional[str] = None,
                           p2p_maddrs: Optional[List[str]] = None, final_stage: bool = False,
                           state: ServerState = ServerState.ONLINE, expiration_time: Optional[float] = None) -> bool:
    exp = expiration_time if expiration_time is not None else get_dht_time() + 90
    rec = {"peer_id": str(peer_id), "timestamp": get_dht_time(), "start_block": int(start_block),
           "end_block": int(end_block), "throughput": float(throughput), "state": state.value,
           "server_address": server_address, "p2p_maddrs": list(p2p_maddrs or []), "final_stage": bool(final_stage)}
    try:
        return dht.store(get_server_key(peer_id, model_name), rec, exp)
    except Exception as e:  # pragma: no cover
        logger.error(f"register_server_on_dht failed: {e}")
        return False


def register_blocks_on_dht(dht: DHT, peer_id, block_indices: List[int], model_name: str = "default",
                           p2p_maddrs: Optional[List[str]] = None, start_block: Optional[int] = None,
                           end_block: Optional[int] = None, throughput: Optional[float] = None,
                           final_stage: bool = False, state: ServerState = ServerState.ONLINE,
                           expiration_time: Optional[float] = None, extra: Optional[dict] = None) -> bool:
    """``extra``: additional record fields (e.g. ``channel_host`` / ``device`` of a server that
    accepts same-node device channels)."""
    exp = expiration_time if expiration_time is not None else get_dht_time() + 90
    try:
        for b in block_indices:
            rec = {"peer_id": str(peer_id), "timestamp": get_dht_time(), "block_idx": int(b),
                   "start_block": None if start_block is None else int(start_block),
                   "end_block": None if end_block is None else int(end_block),
                   "throughput": None if throughput is None else float(throughput), "state": state.value,
                   "p2p_maddrs": list(p2p_maddrs or []), "final_stage": bool(final_stage)}
            if extra:
                rec.update(extra)
            dht.store(get_module_key(b, model_name), rec, exp, subkey=str(peer_id))
        return True
    except Exception as e:  # pragma: no cover
        logger.error(f"register_blocks_on_dht failed: {e}")
        return False


def _unwrap(v: Any) -> Any:
    if hasattr(v, "value"):
        return v.value
    if isinstance(v, tuple) and v:
        return v[0]
    return v


def get_module_entries(dht: DHT, block_idx: int, model_name: str = "default") -> Dict[str, dict]:
    res = dht.get(get_module_key(block_idx, model_name), latest=True)
    if res is None or not isinstance(res.value, dict):
        return {}
    out = {}
    for sk, raw in res.value.items():
        e = _unwrap(raw)
        if isinstance(e, dict):
            out[str(e.get("peer_id") or sk)] = e
    return out


def get_remote_module_infos(dht: DHT, model_name: str = "default",
                            total_blocks: Optional[int] = None) -> List[RemoteModuleInfo]:
    total_blocks = 64 if total_blocks is None else total_blocks
    infos: List[RemoteModuleInfo] = []
    servers: Dict[str, ServerInfo] = {}
    for b in range(total_blocks):
        for pid, e in get_module_entries(dht, b, model_name).items():
            if e.get("start_block") is None or e.get("end_block") is None:
                continue
            if pid not in servers:
                try:
                    st = ServerState(e.get("state", "online"))
                except ValueError:
                    st = ServerState.ONLINE
                servers[pid] = ServerInfo(pid, st, float(e.get("throughput") or 0.0), int(e["start_block"]),
                                          int(e["end_block"]))
            infos.append(RemoteModuleInfo(f"block_{b}", servers[pid]))
    logger.info(f"Retrieved {len(infos)} module infos from registry (total_blocks={total_blocks})")
    return infos


MODELS_KEY = "_petals.models"


def register_model_on_dht(dht: DHT, model_name: str, num_blocks: int, repository: Optional[str] = None,
                          public_name: Optional[str] = None, ttl: float = DEFAULT_TTL) -> bool:
    """Announce which model the swarm serves (upstream ModuleAnnouncerThread stores
    ``_petals.models`` -> {dht_prefix: model info}, petals/server/server.py:674-767), so a client
    can list models without knowing block keys."""
    rec = {"dht_prefix": model_name, "num_blocks": int(num_blocks), "repository": repository or model_name,
           "public_name": public_name, "timestamp": get_dht_time()}
    return dht.store(MODELS_KEY, rec, get_dht_time() + ttl, subkey=model_name)


def get_models_on_dht(dht: DHT) -> Dict[str, dict]:
    res = dht.get(MODELS_KEY, latest=True)
    if res is None or not isinstance(res.value, dict):
        return {}
    return {str(k): _unwrap(v) for k, v in res.value.items() if isinstance(_unwrap(v), dict)}


def update_server_throughput_on_dht(dht: DHT, peer_id, new_throughput: float, model_name: str = "default",
                                    expiration_time: Optional[float] = None) -> bool:
    res = dht.get(get_server_key(peer_id, model_name), latest=True)
    if res is None or not isinstance(res.value, dict):
        return False
    rec = dict(res.value)
    rec["throughput"] = float(new_throughput)
    rec["timestamp"] = get_dht_time()
    exp = expiration_time if expiration_time is not None else get_dht_time() + 90
    return dht.store(get_server_key(peer_id, model_name), rec, exp)

"""boxmot_amd — MI355X-native per-frame association engine for BoxMOT trackers.

Drop-in surface: ``create_tracker``, ``get_tracker_config``, ``ByteTrack``, ``BotSort``, ``OcSort``, ``BoostTrack``, ``StrongSort`` with the
reference's ``update(dets, img, embs) -> [M, 8]`` contract.  The numerics run in libbxassoc.so
(HIP, gfx950); ``boxmot_amd.engine.Engine`` / ``OcsortEngine`` / ``BoostEngine`` / ``SsEngine`` expose the batched many-sequence API.
"""
from .tracker_zoo import create_tracker, get_tracker_config
from .trackers import BoostTrack, BotSort, ByteTrack, OcSort, StrongSort

__version__ = "0.1.0"
__all__ = ["create_tracker", "get_tracker_config", "ByteTrack", "BotSort", "OcSort",
           "BoostTrack", "StrongSort", "__version__"]

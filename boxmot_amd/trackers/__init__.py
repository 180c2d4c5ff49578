from .boosttrack import BoostTrack
from .botsort import BotSort
from .bytetrack import ByteTrack
from .ocsort import OcSort
from .strongsort import StrongSort

__all__ = ["ByteTrack", "BotSort", "OcSort", "BoostTrack", "StrongSort"]

from .botsort import BotSort
from .bytetrack import ByteTrack

__all__ = ["ByteTrack", "BotSort"]

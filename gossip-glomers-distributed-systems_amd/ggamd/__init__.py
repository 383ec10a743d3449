"""ggamd — host side of the MI355X gossip-propagation engine (ctypes over gossip.h)."""
from .engine import Engine, GGError, Topology, load_library, HIP_LIB, HOST_LIB  # noqa: F401

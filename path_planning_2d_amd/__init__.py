"""MI355X-native data-parallel core of the path_planning_2d POMDP grid planner.

Belief propagation (9-neighbour transition stencil, observation likelihood,
renormalisation) and the MDP / FIB Bellman backups run as hand-written gfx950
HIP kernels in ``libpp2_hip.so`` behind the C ABI ``include/pp2.h``.  This
package is the Python host mirror of that boundary.
"""
from ._lib import Pp2Error, LIB_PATH
from .core import GridContext, ShardGroup, device_count
from .planner import BatchedRollout, QVTreePlanner
from . import maps, synthetic

__all__ = ["GridContext", "ShardGroup", "QVTreePlanner", "BatchedRollout", "device_count", "Pp2Error",
           "LIB_PATH", "maps", "synthetic"]

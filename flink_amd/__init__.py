"""flink_amd -- MI355X-native engine for Flink's keyed event-time window aggregation.

The compute path is libflink_amd.so (hand-written HIP for gfx950 behind the C-ABI in
include/flink_amd.h). This package is the host-side mirror of the reference's operator surface:
  flink_amd.engine      WindowAggregator: thin ctypes binding of the C-ABI (fails loudly without the .so)
  flink_amd.operators   WindowOperator (DataStream) / SlicingWindowProcessor (Table) facades
  flink_amd.assigners   TumblingEventTimeWindows, SlidingEventTimeWindows, EventTimeSessionWindows, SliceAssigners
  flink_amd.keygroups   KeyGroupRangeAssignment (host restatement used for routing decisions)
  flink_amd.distributed key-group-partitioned multi-GPU pipeline over torch.distributed (RCCL)
"""
import importlib

__all__ = ["engine", "operators", "assigners", "keygroups", "distributed", "WindowAggregator"]


def __getattr__(name):
    if name == "WindowAggregator":
        return importlib.import_module("flink_amd.engine").WindowAggregator
    if name in ("engine", "operators", "assigners", "keygroups", "distributed"):
        return importlib.import_module("flink_amd." + name)
    raise AttributeError(name)

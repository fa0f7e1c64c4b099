"""Window assigners with the reference's names and argument checks, compiled to the engine config.

DataStream: TumblingEventTimeWindows  flink-streaming-java/.../assigners/TumblingEventTimeWindows.java:50-105
            SlidingEventTimeWindows   .../assigners/SlidingEventTimeWindows.java:50-110
            EventTimeSessionWindows   .../assigners/EventTimeSessionWindows.java:45-120
Table:      SliceAssigners.tumbling/hopping/cumulative  flink-table-runtime/.../slicing/SliceAssigners.java:60-118
"""
import math
from dataclasses import dataclass


@dataclass(frozen=True)
class WindowSpec:
    window_kind: str          # TUMBLE | SLIDE | CUMULATE | SESSION
    semantics: str            # DATASTREAM | TABLE
    size_ms: int = 0
    slide_ms: int = 0
    offset_ms: int = 0
    gap_ms: int = 0

    def config_kwargs(self):
        return dict(window_kind=self.window_kind, semantics=self.semantics, size_ms=self.size_ms,
                    slide_ms=self.slide_ms, offset_ms=self.offset_ms, gap_ms=self.gap_ms)

    # slicing geometry (SliceAssigners / the engine's slice model)
    @property
    def slice_ms(self):
        if self.window_kind == "TUMBLE":
            return self.size_ms
        if self.window_kind == "SLIDE":
            return math.gcd(self.size_ms, self.slide_ms)
        if self.window_kind == "CUMULATE":
            return self.slide_ms
        return 0


class TumblingEventTimeWindows:
    @staticmethod
    def of(size_ms, offset_ms=0):
        if abs(offset_ms) >= size_ms:
            raise ValueError("TumblingEventTimeWindows parameters must satisfy abs(offset) < size")
        return WindowSpec("TUMBLE", "DATASTREAM", size_ms=size_ms, offset_ms=offset_ms)


class SlidingEventTimeWindows:
    @staticmethod
    def of(size_ms, slide_ms, offset_ms=0):
        if abs(offset_ms) >= slide_ms or size_ms <= 0:
            raise ValueError("SlidingEventTimeWindows parameters must satisfy abs(offset) < slide and size > 0")
        return WindowSpec("SLIDE", "DATASTREAM", size_ms=size_ms, slide_ms=slide_ms, offset_ms=offset_ms)


class EventTimeSessionWindows:
    @staticmethod
    def with_gap(gap_ms):
        if gap_ms <= 0:
            raise ValueError("EventTimeSessionWindows parameters must satisfy 0 < size")
        return WindowSpec("SESSION", "DATASTREAM", gap_ms=gap_ms)


class SliceAssigners:
    @staticmethod
    def tumbling(size_ms, offset_ms=0):
        if size_ms <= 0 or abs(offset_ms) >= size_ms:
            raise ValueError("Tumbling Window parameters must satisfy size > 0 and abs(offset) < size")
        return WindowSpec("TUMBLE", "TABLE", size_ms=size_ms, offset_ms=offset_ms)

    @staticmethod
    def hopping(size_ms, slide_ms, offset_ms=0):
        if size_ms <= 0 or slide_ms <= 0:
            raise ValueError("Hopping Window must satisfy slide > 0 and size > 0")
        if size_ms % slide_ms != 0:
            raise ValueError("Slicing Hopping Window requires size must be an integral multiple of slide")
        return WindowSpec("SLIDE", "TABLE", size_ms=size_ms, slide_ms=slide_ms, offset_ms=offset_ms)

    @staticmethod
    def cumulative(max_size_ms, step_ms, offset_ms=0):
        if max_size_ms <= 0 or step_ms <= 0:
            raise ValueError("Cumulative Window parameters must satisfy maxSize > 0 and step > 0")
        if max_size_ms % step_ms != 0:
            raise ValueError("Cumulative Window requires maxSize must be an integral multiple of step")
        return WindowSpec("CUMULATE", "TABLE", size_ms=max_size_ms, slide_ms=step_ms, offset_ms=offset_ms)

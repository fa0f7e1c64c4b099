"""Window assigners with the reference's names and argument checks, compiled to the engine config.

DataStream: TumblingEventTimeWindows  flink-streaming-java/.../assigners/TumblingEventTimeWindows.java:50-105
            SlidingEventTimeWindows   .../assigners/SlidingEventTimeWindows.java:50-110
            EventTimeSessionWindows   .../assigners/EventTimeSessionWindows.java:45-120
Table:      SliceAssigners.tumbling/hopping/cumulative  flink-table-runtime/.../slicing/SliceAssigners.java:60-118
"""
import math
from dataclasses import dataclass

LONG_MAX = (1 << 63) - 1
HOUR_MS = 3_600_000


def _jrem(a, b):
    """Java's % on longs (the sign follows the dividend)."""
    r = abs(a) % abs(b)
    return r if a >= 0 else -r


def window_start_with_offset(timestamp, offset, window_size):
    """TimeWindow.getWindowStartWithOffset (TimeWindow.java:264-272)."""
    return timestamp - _jrem(timestamp - offset + window_size, window_size)


# Shift time zones as the engine takes them (fwa_config.tz): ascending (utc_instant, offset) pairs, the zone's
# ZoneRules transitions (flink_amd/csrc/java_math.h tz_* restated for the host-side operator mirror).
def _tz_offset_at(tz, instant):
    lo, hi = 0, len(tz) - 1
    while lo < hi:
        mid = (lo + hi + 1) >> 1
        if tz[mid][0] <= instant:
            lo = mid
        else:
            hi = mid - 1
    return tz[lo][1]


def to_utc_timestamp_mills(epoch, tz=None):
    """TimeWindowUtil.toUtcTimestampMills: an instant's local wall-clock time as UTC epoch millis (:52-60)."""
    if not tz or epoch == LONG_MAX:
        return epoch
    return epoch + _tz_offset_at(tz, epoch)


def _at_zone(tz, local):
    j = 0
    lo, hi = 1, len(tz) - 1
    while lo <= hi:
        mid = (lo + hi) >> 1
        if tz[mid][0] + tz[mid][1] <= local:
            j, lo = mid, mid + 1
        else:
            hi = mid - 1
    if j > 0 and local < tz[j][0] + tz[j - 1][1]:
        return local - tz[j - 1][1]                   # overlap: the earlier offset
    return local - tz[j][1]


def to_epoch_mills_for_timer(local, tz=None):
    """TimeWindowUtil.toEpochMillsForTimer (:74-95): the instant a local window time triggers at (DST gap: the
    hour's start; overlap: the later instant)."""
    if not tz or local == LONG_MAX:
        return local
    if len(tz) == 1:
        return local - tz[0][1]
    t1, t2 = _at_zone(tz, local), _at_zone(tz, local + HOUR_MS)
    if t1 == t2:
        return t1 - _jrem(t1, HOUR_MS)
    if t2 - t1 > HOUR_MS:
        return t1 + HOUR_MS
    return t1


def is_window_fired(window_end, current_progress, tz=None):
    """TimeWindowUtil.isWindowFired (:175-183)."""
    if window_end == LONG_MAX:
        return False
    return current_progress >= to_epoch_mills_for_timer(window_end - 1, tz)


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

    # Table slice assigners (SliceAssigners.java:160-335): the slice a (local) timestamp falls in and the end of the
    # last window containing that slice
    def assign_slice_end(self, timestamp):
        step = self.slice_ms
        return window_start_with_offset(timestamp, self.offset_ms, step) + step

    def last_window_end(self, slice_end):
        if self.window_kind == "TUMBLE":
            return slice_end
        if self.window_kind == "SLIDE":
            return slice_end - self.slice_ms + self.size_ms
        if self.window_kind == "CUMULATE":
            return window_start_with_offset(slice_end - 1, self.offset_ms, self.size_ms) + self.size_ms
        raise ValueError("no slices for %s windows" % self.window_kind)

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

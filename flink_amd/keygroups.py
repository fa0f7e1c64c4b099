"""KeyGroupRangeAssignment restated for host-side routing decisions (which rank owns which key groups).

flink-runtime/src/main/java/org/apache/flink/runtime/state/KeyGroupRangeAssignment.java:
  computeKeyGroupRangeForOperatorIndex :93-106, computeOperatorIndexForKeyGroup :124-127.
Per-record key-group computation is done on the GPU (flink_amd.engine.key_groups / fwa_key_groups).
"""

DEFAULT_LOWER_BOUND_MAX_PARALLELISM = 1 << 7   # :32
UPPER_BOUND_MAX_PARALLELISM = 1 << 15          # Transformation.java:110


def check_parallelism(p):
    if not (0 < p <= UPPER_BOUND_MAX_PARALLELISM):
        raise ValueError("Operator parallelism not within bounds: %d" % p)


def key_group_range_for_operator(max_parallelism, parallelism, operator_index):
    """(start, end) inclusive range owned by subtask `operator_index`."""
    check_parallelism(parallelism)
    check_parallelism(max_parallelism)
    if max_parallelism < parallelism:
        raise ValueError("Maximum parallelism must not be smaller than parallelism.")
    start = (operator_index * max_parallelism + parallelism - 1) // parallelism
    end = ((operator_index + 1) * max_parallelism - 1) // parallelism
    return start, end


def operator_index_for_key_group(max_parallelism, parallelism, key_group):
    return key_group * parallelism // max_parallelism

"""Config C1 (BASELINE.json configs[0]): the WindowWordCount example's count windows, CPU by design.

SURVEY.md §8(a) a22 marks this path "Not GPU": count windows over String keys are plumbing, restated
here at parallelism 1 so a user of the reference finds the example's behaviour. It is not a fallback
of the GPU engine (the event-time window path has none).

Reference chain:
  WindowWordCount.main          flink-examples-streaming/.../windowing/WindowWordCount.java
    flatMap(WordCount.Tokenizer)  .../wordcount/WordCount.java:171-186  (lower-case, split on \\W+)
    keyBy(f0).countWindow(size, slide)  KeyedStream.java:734-738
       = GlobalWindows + CountEvictor.of(size) + CountTrigger.of(slide) -> EvictingWindowOperator
         (WindowOperatorBuilder.java:286-300)
    .sum(1)                       SumAggregator.reduce (SumAggregator.java:66-76)
  CountTrigger.onElement          CountTrigger.java:47-56: per-key counter += 1; at >= slide -> clear, FIRE
  CountEvictor.evictBefore        CountEvictor.java:65-81: keep the last `size` elements (evicted ones
                                  are removed from the window state for good)
  FIRE (not PURGE): the list state keeps the retained elements for the next firing.
"""
import re
from collections import defaultdict

_SPLIT = re.compile(r"\W+", re.ASCII)   # Java "\\W+" is ASCII-only: [^a-zA-Z0-9_]+ (WordCount.java:171-186)


def tokenize(line):
    """WordCount.Tokenizer.flatMap: (token, 1) for every non-empty token of the lower-cased line."""
    return [(t, 1) for t in _SPLIT.split(line.lower()) if t]


class CountWindowSum:
    """keyBy(word).countWindow(size, slide).sum(1) at parallelism 1 (EvictingWindowOperator)."""

    def __init__(self, size=250, slide=150):
        if size <= 0 or slide <= 0:
            raise ValueError("window size and slide must be positive")
        self.size, self.slide = size, slide
        self.contents = defaultdict(list)   # ListState of the GlobalWindow per key
        self.count = defaultdict(int)       # CountTrigger's ReducingState counter per key

    def process_element(self, key, value):
        """Returns the emitted (key, sum) tuple when this element fires the key's window, else None."""
        elems = self.contents[key]
        elems.append(value)
        self.count[key] += 1
        if self.count[key] < self.slide:
            return None
        self.count[key] = 0                              # CountTrigger: clear, FIRE
        if len(elems) > self.size:                       # CountEvictor.evictBefore
            del elems[: len(elems) - self.size]
        return key, sum(elems)                           # SumAggregator over the retained elements


def window_word_count(lines, size=250, slide=150):
    """Run the example over text lines; returns the emitted (word, count) tuples in emission order."""
    op = CountWindowSum(size, slide)
    out = []
    for line in lines:
        for word, one in tokenize(line):
            r = op.process_element(word, one)
            if r is not None:
                out.append(r)
    return out


def format_result(t):
    """Tuple2.toString as written by the example's FileSink (SimpleStringEncoder)."""
    return "(%s,%d)" % t

"""CPU tests for config C1 (WindowWordCount count windows).

StreamingExamplesITCase.testWindowWordCount (window 25, slide 15) only checks that every result line
matches ^\\([a-z]+,(\\d)+\\); the text below is our own (the example's bundled text is not copied). The
count semantics are checked against CountTrigger/CountEvictor directly: a word's k-th firing happens at
its (15k)-th occurrence and reports min(15k, 25).
"""
import re

from flink_amd.count_windows import CountWindowSum, format_result, tokenize, window_word_count

TEXT = ["The quick brown fox jumps over the lazy dog; the dog sleeps, the fox runs.",
        "To be or not to be -- that is the question: whether 'tis nobler in the mind"] * 40


def test_tokenizer_matches_java_split():
    assert tokenize("Hello, World!! foo_bar 42x") == [("hello", 1), ("world", 1), ("foo_bar", 1), ("42x", 1)]
    assert tokenize("  --  ") == []
    # Java's \\W is ASCII-only ([^a-zA-Z0-9_]): non-ASCII letters split tokens (toLowerCase is Unicode)
    assert tokenize("Café Straße ÆON x") == [("caf", 1), ("stra", 1), ("e", 1), ("on", 1), ("x", 1)]


def test_itcase_regexp_and_counts():
    out = window_word_count(TEXT, size=25, slide=15)
    assert out, "no window fired"
    pat = re.compile(r"^\([a-z]+,(\d)+\)")
    assert all(pat.match(format_result(t)) for t in out)
    seen = {}
    for w, c in out:
        k = seen.get(w, 0) + 1
        seen[w] = k
        assert c == min(15 * k, 25), (w, k, c)
    occ = {}
    for line in TEXT:
        for w, _ in tokenize(line):
            occ[w] = occ.get(w, 0) + 1
    assert seen == {w: n // 15 for w, n in occ.items() if n >= 15}


def test_evictor_keeps_last_size_elements():
    op = CountWindowSum(size=3, slide=2)
    got = [op.process_element("k", v) for v in (1, 2, 3, 4, 5, 6)]
    assert got == [None, ("k", 3), None, ("k", 9), None, ("k", 15)]   # [1,2] -> [2,3,4] -> [4,5,6]

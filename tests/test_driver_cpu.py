"""CPU tests of the inference.py driver pieces that are plain host logic (no GPU): the text
preprocessing of StyleTTS2.generate (reference inference.py:17-42, 50-55), TextCleaner
(meldataset.py:21-35) and the 20-s reference-audio cap of __compute_style (inference.py:180-188).
Expected values are worked by hand from the reference source (nltk / librosa are absent here)."""
import numpy as np

from stts2_mi355x.inference import MAX_REF_SAMPLES, Preprocess, TextCleaner


def test_text_normalize_maps_punctuation_and_whitespace():
    p = Preprocess()
    assert p.text_normalize("  a, b;c (d)  e?\tf…g!h:i–j。k  ") == "a, b.c .d) e. f.g.h.i.j.k"


def test_text_preprocess_splits_and_merges():
    p = Preprocess()
    text = "one two three four. five six seven eight nine. ten; eleven"
    # sentences: [4 words], [5 words], [1], [1] -> n=4: "one..four" | "five..nine" | "ten, eleven" (2 words)
    # -> the short last merges into the one before it
    assert p.text_preprocess(text, n_merge=4) == ["one two three four", "five six seven eight nine, ten, eleven"]
    assert p.text_preprocess("a. b. c", n_merge=12) == ["a, b, c"]
    assert p.text_preprocess("single sentence without a period", n_merge=2) == ["single sentence without a period"]
    assert p.text_preprocess(" .. ", n_merge=3) == []


def test_merge_fragments_reference_cases():
    m = Preprocess.merge_fragments
    assert m(["a b", "c", "d e f"], 3) == ["a b, c", "d e f"]
    assert m(["a b c", "d"], 3) == ["a b c, d"]
    assert m(["a"], 3) == ["a"]


def test_text_cleaner_skips_unknown():
    c = TextCleaner({"a": 1, "b": 2, " ": 3})
    assert c("ab ba?x") == [1, 2, 3, 2, 1]


def test_reference_audio_cap_constant():
    assert MAX_REF_SAMPLES == 24000 * 20
    # get_style caps before chunking: a 25-s clip chunks as the first 20 s do (6 full 3-s chunks,
    # the 2-s tail counts) -- the arithmetic of inference.py:195-217 on 480,000 samples
    total, jump = MAX_REF_SAMPLES, 3 * 24000
    full = [0] + [i for i in range(jump, total, jump) if i + jump < total]
    tail = [i for i in range(jump, total, jump) if i + jump >= total and (total - i) / 24000 >= 1]
    assert len(full) == 6 and len(tail) == 1
    assert np.isclose((total - tail[0]) / 24000, 2.0)

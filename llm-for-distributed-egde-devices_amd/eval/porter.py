"""Porter stemmer (Porter 1980), used by ROUGE with ``use_stemmer=True``.

The reference scores ROUGE through ``rouge_score.RougeScorer([...], use_stemmer=True)``
(combine_model_fp_updated.py:46), which stems with NLTK's PorterStemmer (default
NLTK_EXTENSIONS mode).  Neither package is installed here, so this is an independent
implementation of the algorithm including the NLTK-extension behaviours that matter for
English prose: words of <= 2 letters are left alone, the irregular-forms table, step 1c only
rewrites y->i after a consonant, and step 2's extra ``logi``/``fulli``/``lessli`` rules.
Parity note: stems of rare words may differ from NLTK in corner cases ("parity unpinned").
"""
from __future__ import annotations

_IRREGULAR = {
    "skies": "sky", "sky": "sky", "dying": "die", "lying": "lie", "tying": "tie", "news": "news",
    "innings": "inning", "inning": "inning", "outings": "outing", "outing": "outing", "cannings": "canning",
    "canning": "canning", "howe": "howe", "proceed": "proceed", "exceed": "exceed", "succeed": "succeed",
}
_VOWELS = frozenset("aeiou")


def _cons(w: str, i: int) -> bool:
    c = w[i]
    if c in _VOWELS:
        return False
    if c == "y":
        return i == 0 or not _cons(w, i - 1)
    return True


def _m(stem: str) -> int:
    """Number of VC sequences in the stem."""
    n, i, L = 0, 0, len(stem)
    while i < L and _cons(stem, i):
        i += 1
    while i < L:
        while i < L and not _cons(stem, i):
            i += 1
        if i >= L:
            break
        n += 1
        while i < L and _cons(stem, i):
            i += 1
    return n


def _has_vowel(stem: str) -> bool:
    return any(not _cons(stem, i) for i in range(len(stem)))


def _double_cons(w: str) -> bool:
    return len(w) >= 2 and w[-1] == w[-2] and _cons(w, len(w) - 1)


def _cvc(w: str) -> bool:
    if len(w) < 3:
        return False
    return (_cons(w, len(w) - 3) and not _cons(w, len(w) - 2) and _cons(w, len(w) - 1)
            and w[-1] not in "wxy")


def _replace(w: str, rules, cond) -> str:
    for suf, rep in rules:
        if w.endswith(suf):
            stem = w[: len(w) - len(suf)]
            return stem + rep if cond(stem) else w
    return w


_STEP2 = [("ational", "ate"), ("tional", "tion"), ("enci", "ence"), ("anci", "ance"), ("izer", "ize"),
          ("bli", "ble"), ("alli", "al"), ("entli", "ent"), ("eli", "e"), ("ousli", "ous"), ("ization", "ize"),
          ("ation", "ate"), ("ator", "ate"), ("alism", "al"), ("iveness", "ive"), ("fulness", "ful"),
          ("ousness", "ous"), ("aliti", "al"), ("iviti", "ive"), ("biliti", "ble"), ("fulli", "ful"),
          ("lessli", "less"), ("logi", "log")]
_STEP3 = [("icate", "ic"), ("ative", ""), ("alize", "al"), ("iciti", "ic"), ("ical", "ic"), ("ful", ""),
          ("ness", "")]
_STEP4 = ["al", "ance", "ence", "er", "ic", "able", "ible", "ant", "ement", "ment", "ent", "ion", "ou", "ism",
          "ate", "iti", "ous", "ive", "ize"]


def stem(word: str) -> str:
    w = word.lower()
    if w in _IRREGULAR:
        return _IRREGULAR[w]
    if len(w) <= 2:
        return w
    # step 1a
    if w.endswith("sses"):
        w = w[:-2]
    elif w.endswith("ies"):
        w = w[:-3] + ("ie" if len(w) == 4 else "i")
    elif w.endswith("ss"):
        pass
    elif w.endswith("s"):
        w = w[:-1]
    # step 1b
    extra = False
    if w.endswith("eed"):
        if _m(w[:-3]) > 0:
            w = w[:-1]
    elif w.endswith("ed") and _has_vowel(w[:-2]):
        w, extra = w[:-2], True
    elif w.endswith("ing") and _has_vowel(w[:-3]):
        w, extra = w[:-3], True
    if extra:
        if w.endswith(("at", "bl", "iz")):
            w += "e"
        elif _double_cons(w) and w[-1] not in "lsz":
            w = w[:-1]
        elif _m(w) == 1 and _cvc(w):
            w += "e"
    # step 1c (NLTK: only after a consonant, stem longer than one letter)
    if w.endswith("y") and len(w) > 2 and _cons(w, len(w) - 2):
        w = w[:-1] + "i"
    # step 2, 3
    w = _replace(w, _STEP2, lambda s: _m(s) > 0)
    w = _replace(w, _STEP3, lambda s: _m(s) > 0)
    # step 4
    for suf in sorted(_STEP4, key=len, reverse=True):
        if w.endswith(suf):
            s = w[: len(w) - len(suf)]
            if _m(s) > 1 and (suf != "ion" or (s and s[-1] in "st")):
                w = s
            break
    # step 5a
    if w.endswith("e"):
        s = w[:-1]
        if _m(s) > 1 or (_m(s) == 1 and not _cvc(s)):
            w = s
    # step 5b
    if _m(w) > 1 and _double_cons(w) and w.endswith("l"):
        w = w[:-1]
    return w

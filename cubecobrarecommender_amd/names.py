"""Card-name normalisation: ``unidecode.unidecode(name.lower())`` (src/scripts/ml_recommend.py:44,
web/ml_recommend_web.py:29).  ``unidecode`` (requirements.txt:53) is not installed in this
pipeline, so this is a restatement for the characters card names use: NFKD decomposition with
combining marks dropped, plus unidecode's transliterations of the non-decomposable Latin letters.
SURVEY §8(f) row N3; strings outside this table keep their characters (parity unpinned).
"""
import unicodedata

_SPECIAL = {
    'æ': 'ae', 'Æ': 'AE', 'œ': 'oe', 'Œ': 'OE', 'ß': 'ss', 'ø': 'o', 'Ø': 'O', 'đ': 'd', 'Đ': 'D',
    'ð': 'd', 'Ð': 'D', 'þ': 'th', 'Þ': 'Th', 'ł': 'l', 'Ł': 'L', 'ı': 'i', 'ŋ': 'ng', 'ĸ': 'q',
    '‘': "'", '’': "'", '‚': ',', '“': '"', '”': '"', '–': '-', '—': '-', '…': '...', ' ': ' ',
    '™': '(tm)', '®': '(r)', '©': '(c)', '½': ' 1/2', '×': 'x', '−': '-',
}


def unidecode_lite(s):
    out = []
    for ch in unicodedata.normalize('NFKD', s):
        if unicodedata.combining(ch):
            continue
        out.append(_SPECIAL.get(ch, ch))
    return ''.join(out)


def normalize(name):
    """The lookup key of ml_recommend.py:44: unidecode(name.lower())."""
    return unidecode_lite(name.lower())

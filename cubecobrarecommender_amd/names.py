"""Card-name normalisation: ``unidecode.unidecode(name.lower())`` (src/scripts/ml_recommend.py:44,
web/ml_recommend_web.py:29; the same key in src/scripts/recommend.py:53 and cut_cards.py:53).

``Unidecode==1.1.1`` (requirements.txt:53) is not installed in this pipeline, so its algorithm is
restated here:

* a code point below 0x80 is itself;
* otherwise unidecode looks up ``x{cp >> 8:03x}.data[cp & 0xFF]`` — one replacement string per
  code point, '' where the table holds none (its default ``errors='ignore'``);
* code points above 0xEFFFF (private use and beyond) map to ''.

The tables are restated for the blocks card names and their typographic variants use: Latin-1
Supplement (x000), Latin Extended-A (x001), the Latin Extended-B letters with a plain base, Greek
(x003, basic letters), Cyrillic (x004, basic letters), General Punctuation (x020), Letterlike
Symbols / Number Forms (x021: the (tm)-style and Roman-numeral entries), and for the Korean and
Japanese printings: the Hangul syllables (xac..xd7, which unidecode's tables spell out as the
syllable's initial + medial + final jamo romanisation — generated here from the same three
lists) and the hiragana / katakana of x030 (Kunrei-style: si, ti, tu, hu; small kana as their
full-size letter; the prolonged-sound mark '-').  A code point outside them is decomposed (NFKD)
and its base letters looked up the same way — that matches unidecode for the accented letters of
other Latin blocks (x01e: Vietnamese etc.).  What none covers (CJK ideographs, whose unidecode
tables give pinyin with a trailing space, and other scripts) keeps its characters, so such a name
simply misses the id map: parity unpinned everywhere outside ASCII (no reference output exists
in this pipeline: the reference's ml_files/*_id_map.json are Git-LFS pointers).
"""
import unicodedata

# x000: U+0080..U+00FF (C1 controls -> '')
_X000 = (
    [''] * 32 +
    [' ', '!', 'C/', 'PS', '$?', 'Y=', '|', 'SS', '"', '(c)', 'a', '<<', '!', '', '(r)', '-',
     'deg', '+-', '2', '3', "'", 'u', 'P', '*', ',', '1', 'o', '>>', ' 1/4', ' 1/2', ' 3/4', '?',
     'A', 'A', 'A', 'A', 'A', 'A', 'AE', 'C', 'E', 'E', 'E', 'E', 'I', 'I', 'I', 'I',
     'D', 'N', 'O', 'O', 'O', 'O', 'O', 'x', 'O', 'U', 'U', 'U', 'U', 'Y', 'Th', 'ss',
     'a', 'a', 'a', 'a', 'a', 'a', 'ae', 'c', 'e', 'e', 'e', 'e', 'i', 'i', 'i', 'i',
     'd', 'n', 'o', 'o', 'o', 'o', 'o', '/', 'o', 'u', 'u', 'u', 'u', 'y', 'th', 'y'])
assert len(_X000) == 128

# x001 part 1: U+0100..U+017F (Latin Extended-A)
_X001A = ('A a A a A a C c C c C c C c D d D d E e E e E e E e E e G g G g G g G g H h H h '
          'I i I i I i I i I i IJ ij J j K k q L l L l L l L l L l N n N n N n \'n NG ng '
          'O o O o O o OE oe R r R r R r S s S s S s S s T t T t T t U u U u U u U u U u U u '
          'W w Y y Y Z z Z z Z z s').split(' ')
assert len(_X001A) == 128

# Greek (x003): basic capital and small letters, tonos forms
_GREEK = {}
for caps, small, lat in zip('ΑΒΓΔΕΖΗΘΙΚΛΜΝΞΟΠΡΣΤΥΦΧΨΩ', 'αβγδεζηθικλμνξοπρστυφχψω',
                            ['A', 'B', 'G', 'D', 'E', 'Z', 'E', 'Th', 'I', 'K', 'L', 'M', 'N', 'Ks',
                             'O', 'P', 'R', 'S', 'T', 'U', 'Ph', 'Kh', 'Ps', 'O']):
    _GREEK[caps] = lat
    _GREEK[small] = lat.lower()
_GREEK.update({'ς': 's', 'ά': 'a', 'έ': 'e', 'ή': 'e', 'ί': 'i', 'ό': 'o', 'ύ': 'u', 'ώ': 'o',
               'Ά': 'A', 'Έ': 'E', 'Ή': 'E', 'Ί': 'I', 'Ό': 'O', 'Ύ': 'U', 'Ώ': 'O', 'ϊ': 'i', 'ϋ': 'u',
               'ΐ': 'i', 'ΰ': 'u', 'Ϊ': 'I', 'Ϋ': 'U'})

# Cyrillic (x004): U+0410..U+044F plus Ё / ё
_CYR = {}
for i, lat in enumerate(['A', 'B', 'V', 'G', 'D', 'E', 'Zh', 'Z', 'I', 'I', 'K', 'L', 'M', 'N', 'O', 'P',
                         'R', 'S', 'T', 'U', 'F', 'Kh', 'Ts', 'Ch', 'Sh', 'Shch', "'", 'Y', "'", 'E', 'Iu', 'Ia']):
    _CYR[chr(0x410 + i)] = lat
    _CYR[chr(0x430 + i)] = lat.lower()
_CYR.update({'Ё': 'Io', 'ё': 'io'})

# General Punctuation (x020) and Letterlike Symbols / Number Forms (x021) entries names use
_PUNCT = {
    ' ': ' ', ' ': ' ', ' ': ' ', ' ': ' ', ' ': ' ', ' ': ' ', ' ': ' ',
    ' ': ' ', ' ': ' ', ' ': ' ', ' ': ' ', '​': '', '‌': '', '‍': '',
    '‐': '-', '‑': '-', '‒': '-', '–': '-', '—': '--', '―': '--',
    '‖': '||', '‗': '_', '‘': "'", '’': "'", '‚': ',', '‛': "'",
    '“': '"', '”': '"', '„': ',,', '‟': '"', '†': '+', '‡': '++',
    '•': '*', '‣': '*>', '․': '.', '‥': '..', '…': '...', '‧': '.',
    ' ': ' ', '‰': '%0', '′': "'", '″': "''", '‹': '<', '›': '>',
    '⁄': '/', '™': '(tm)', '№': 'No', '←': '<-', '→': '->',
    'ʼ': "'", 'ˆ': '^', '˜': '~', '−': '-',
}
for i, r in enumerate(['I', 'II', 'III', 'IV', 'V', 'VI', 'VII', 'VIII', 'IX', 'X', 'XI', 'XII', 'L', 'C', 'D', 'M']):
    _PUNCT[chr(0x2160 + i)] = r
    _PUNCT[chr(0x2170 + i)] = r.lower()

# Hangul syllables U+AC00..U+D7A3 = 0xAC00 + (initial * 21 + medial) * 28 + final
_HANGUL_INITIAL = ['g', 'gg', 'n', 'd', 'dd', 'r', 'm', 'b', 'bb', 's', 'ss', '', 'j', 'jj', 'c', 'k', 't', 'p', 'h']
_HANGUL_MEDIAL = ['a', 'ae', 'ya', 'yae', 'eo', 'e', 'yeo', 'ye', 'o', 'wa', 'wae', 'oe', 'yo', 'u', 'weo', 'we',
                  'wi', 'yu', 'eu', 'yi', 'i']
_HANGUL_FINAL = ['', 'g', 'gg', 'gs', 'n', 'nj', 'nh', 'd', 'l', 'lg', 'lm', 'lb', 'ls', 'lt', 'lp', 'lh', 'm',
                 'b', 'bs', 's', 'ss', 'ng', 'j', 'c', 'k', 't', 'p', 'h']


def _hangul(cp):
    i = cp - 0xAC00
    return _HANGUL_INITIAL[i // (21 * 28)] + _HANGUL_MEDIAL[(i // 28) % 21] + _HANGUL_FINAL[i % 28]


# x030: hiragana U+3041..U+3094 (katakana U+30A1..U+30F4 are the same syllables + 0x60)
_KANA = ('a a i i u u e e o o ka ga ki gi ku gu ke ge ko go sa za si zi su zu se ze so zo ta da ti di tu tu du '
         'te de to do na ni nu ne no ha ba pa hi bi pi hu bu pu he be pe ho bo po ma mi mu me mo ya ya yu yu '
         'yo yo ra ri ru re ro wa wa wi we wo n vu').split(' ')
assert len(_KANA) == 0x3094 - 0x3041 + 1
_JP = {chr(0x3041 + i): r for i, r in enumerate(_KANA)}
_JP.update({chr(0x30A1 + i): r for i, r in enumerate(_KANA)})
_JP.update({'ヵ': 'ka', 'ヶ': 'ke', 'ヷ': 'va', 'ヸ': 'vi', 'ヹ': 've', 'ヺ': 'vo', 'ー': '-', '・': '*',
            '　': ' ', '、': ',', '。': '.', '「': '[', '」': ']', '『': '[[', '』': ']]'})

_TABLE = {chr(0x80 + i): r for i, r in enumerate(_X000)}
_TABLE.update({chr(0x100 + i): r for i, r in enumerate(_X001A)})
_TABLE.update(_GREEK)
_TABLE.update(_CYR)
_TABLE.update(_PUNCT)
_TABLE.update(_JP)


def _repl(ch):
    cp = ord(ch)
    if cp < 0x80:
        return ch
    if cp > 0xEFFFF:
        return ''
    r = _TABLE.get(ch)
    if r is not None:
        return r
    if 0xAC00 <= cp <= 0xD7A3:
        return _hangul(cp)
    # other blocks: NFKD base letters, each looked up again (combining marks -> '')
    dec = unicodedata.normalize('NFKD', ch)
    if dec != ch:
        return ''.join('' if unicodedata.combining(c) else _repl(c) for c in dec)
    if unicodedata.combining(ch):
        return ''
    return ch   # not restated (CJK, other scripts): parity unpinned, see the module docstring


def unidecode(s):
    """unidecode.unidecode (Unidecode 1.1.1) for the blocks restated above."""
    if s.isascii():
        return s
    return ''.join(_repl(ch) for ch in s)


def normalize(name):
    """The lookup key of ml_recommend.py:44: unidecode(name.lower())."""
    return unidecode(name.lower())

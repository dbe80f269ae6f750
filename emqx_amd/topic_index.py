"""Host mirror of `emqx_topic_index` (apps/emqx/src/emqx_topic_index.erl:21-32) over the
MI355X engine.

Same names, argument meaning and error behaviour as the reference module, so the
reference's suite (apps/emqx/test/emqx_topic_index_SUITE.erl) reads the same:

    tab = TopicIndex.new()
    tab.insert(b"sensor/+/#", "t_insert_2", b"")      # insert/4
    tab.matches(b"sensor/1", [])                      # matches/3 -> [Key]
    tab.match(b"sensor")                              # match/2 -> Key | False
    get_id(key), get_topic(key), tab.get_record(key)

A key is the reference's `{Filter, {ID}}`: `(words_tuple | bytes, (ID,))`.  Writes are
visible to the next read (ETS semantics for one caller): they are staged in the
engine and committed as one delta epoch before the next match.  `matches_batch`
is the batched entry point the GPU exists for.

IDs may be any hashable Erlang-like term (int, str-as-atom, tuple, bytes); the
engine sees a dense u64 per distinct ID and the mirror maps back.
"""
from __future__ import annotations

from . import _native as N
from .topic import HASH, PLUS, filter_words, join, term_key, wildcard


class BadArg(ValueError):
    """error(badarg): a topic level is exactly '+' or '#' (emqx_trie_search.erl:374-375)."""


def make_key(topic_or_words, ident):
    """emqx_trie_search:make_key/2 (emqx_trie_search.erl:115-128)."""
    if isinstance(topic_or_words, (list, tuple)):
        return (tuple(topic_or_words), (ident,))
    ws = filter_words(topic_or_words)
    if wildcard(ws):
        return (tuple(ws), (ident,))
    return (bytes(topic_or_words) if not isinstance(topic_or_words, str) else topic_or_words.encode(), (ident,))


def get_id(key):
    """emqx_topic_index:get_id/1."""
    return key[1][0]


def get_topic(key):
    """emqx_topic_index:get_topic/1: join the words of a list key, or the binary."""
    f = key[0]
    return join(list(f)) if isinstance(f, tuple) else f


def _key_order(key):
    f, (ident,) = key
    fk = term_key(list(f)) if isinstance(f, tuple) else term_key(f)
    return (fk, term_key(ident))


def words_topic_bytes(words) -> bytes:
    """A pre-split topic (matches/3 takes `[word()]`, emqx_trie_search.erl:182,369-370) as
    the bytes of a topic filter with the same walk.  A word list is used as is: no badarg
    check, so '+' / '#' atoms act as wildcards of the topic (compare/3's filter-search
    clauses, :292-300), and the final match_topics/4 step (:381-389) adds nothing, since a
    list never equals or sorts above a binary key: a word-list topic matches exactly what
    matches_filter/3 of the same words matches.

    Words the byte form cannot carry are refused (ValueError): one containing '/', and the
    binaries <<"+">> / <<"#">> (plain words in a list, wildcards once joined).  Standing in
    another word for them is not exact: the reference's walk decides `lower` (stop) by the
    term order of the words (:325-332), so the stand-in would have to sort exactly where the
    original does among the index's words."""
    out = []
    for w in words:
        if isinstance(w, str) and w in (PLUS, HASH):  # the atoms
            out.append(w.encode())
            continue
        wb = w.encode() if isinstance(w, str) else bytes(w)
        if b"/" in wb or wb in (b"+", b"#"):
            raise ValueError(f"word {wb!r} has no byte form (contains '/' or is a binary '+'/'#')")
        out.append(wb)
    return b"/".join(out)


class TopicIndex:
    def __init__(self, device: int = 0, engine: N.Engine | None = None, **engine_kw):
        self.eng = engine or N.Engine(device, **engine_kw)
        self._ids: dict = {}        # term -> u64
        self._terms: list = []      # u64 -> term
        self._records: dict = {}    # key -> record
        self._dirty = False
        self._max_word = 0          # longest filter word ever inserted (word-list topics)

    @classmethod
    def new(cls, device: int = 0, **kw) -> "TopicIndex":
        return cls(device, **kw)

    # ---- id mapping
    def _id(self, term) -> int:
        u = self._ids.get(term)
        if u is None:
            u = len(self._terms)
            self._ids[term] = u
            self._terms.append(term)
        return u

    @staticmethod
    def _filter_bytes(filt):
        """(bytes, flags) handed to the engine for a binary or word-list filter."""
        if isinstance(filt, (list, tuple)):
            ws = list(filt)
            for w in ws:
                if isinstance(w, (bytes, bytearray)) and b"/" in w:
                    raise ValueError("word contains '/'")
            return join(ws), N.TM_KEY_WORDS
        return (filt.encode() if isinstance(filt, str) else bytes(filt)), 0

    # ---- writes: insert/4, delete/3
    def insert(self, filt, ident, record=b"", tab=None) -> bool:
        fb, flags = self._filter_bytes(filt)
        self._max_word = max(self._max_word, max(len(w) for w in fb.split(b"/")))
        self.eng.apply([(N.TM_OP_ADD, fb, self._id(ident), flags)])
        self._records[make_key(filt, ident)] = record
        self._dirty = True
        return True

    def delete(self, filt, ident, tab=None) -> bool:
        fb, flags = self._filter_bytes(filt)
        if ident in self._ids:
            self.eng.apply([(N.TM_OP_DEL, fb, self._ids[ident], flags)])
            self._records.pop(make_key(filt, ident), None)
            self._dirty = True
        return True

    def commit(self):
        if self._dirty:
            self.eng.commit()
            self._dirty = False

    # ---- reads
    def _key_of(self, handle: int):
        u, fb, flags = self.eng.key_info(handle)
        ident = self._terms[u]
        if flags & N.TM_KEY_WORDS or wildcard(filter_words(fb)):
            return (tuple(filter_words(fb)), (ident,))
        return (fb, (ident,))

    def matches_batch(self, topics, opts=()) -> list:
        """Batched matches/3: one list of keys per topic; BadArg instances for
        topics with a '+'/'#' level.  A topic may also be a word list (words_topic_bytes)."""
        self.commit()
        topics = list(topics)
        wl = [i for i, t in enumerate(topics) if isinstance(t, (list, tuple))]
        out = [None] * len(topics)
        if wl:
            empty = [i for i in wl if not topics[i]]
            # lists of binary words: the engine's own walk of word-list topics
            # (TM_MATCH_TOPIC_WORDS); lists holding the '+' / '#' / '' atoms act as filters of
            # the walk (compare/3's filter-search clauses) and go through matches_filter
            plain = [i for i in wl if topics[i] and not any(isinstance(w, str) and w in (PLUS, HASH, "")
                                                           for w in topics[i])
                     and not any(b"/" in (w.encode() if isinstance(w, str) else bytes(w)) for w in topics[i])]
            if plain:
                for i, hs in zip(plain, self.eng.match_words([topics[i] for i in plain], N.TM_MATCH_ALL)):
                    out[i] = self._reduce([self._key_of(h) for h in hs], opts)
            byw = [i for i in wl if topics[i] and out[i] is None]
            if byw:
                for i, r in zip(byw, self.matches_filter_batch([words_topic_bytes(topics[i]) for i in byw], opts)):
                    out[i] = r
            if empty:
                # [] words: only the root '#' filter compares match_full against them (:282-290;
                # every longer filter is `lower`, :333-340); a one-level unknown word reaches
                # exactly '#', '+' and '+/#', of which '#' is kept
                root = self.matches_filter_batch([b"\xff" * (self._max_word + 1)], ())[0]
                keys = [k for k in root if isinstance(k[0], tuple) and k[0] == (HASH,)]
                for i in empty:
                    out[i] = self._reduce(keys, opts)
        rest = [i for i in range(len(topics)) if out[i] is None]
        handles = self.eng.match([topics[i] for i in rest], N.TM_MATCH_ALL) if rest else []
        for i, hs in zip(rest, handles):
            if hs is None:
                out[i] = BadArg("badarg")
                continue
            keys = [self._key_of(h) for h in hs]
            out[i] = self._reduce(keys, opts)
        return out

    @staticmethod
    def _reduce(keys, opts):
        opts = list(opts)
        if "return_first" in opts:
            return [min(keys, key=_key_order)] if keys else []
        if "unique" in opts:
            best = {}
            for k in sorted(keys, key=_key_order):  # ascending walk order: last write wins
                best[get_id(k)] = k
            return [best[i] for i in sorted(best, key=term_key)]
        return keys

    def matches(self, topic, tab=None, opts=()):
        r = self.matches_batch([topic], opts)[0]
        if isinstance(r, BadArg):
            raise r
        return r

    def matches_filter_batch(self, filters, opts=()) -> list:
        """Batched matches_filter/3 (emqx_topic_index.erl:82-84): one list of keys per topic
        filter, in the reference's list order (its accumulator: the walk's keys reversed,
        i.e. descending term order).  BadArg for a filter with '#' before its last level
        (the reference's walk never returns on one)."""
        self.commit()
        out = []
        for hs in self.eng.match_filter(filters, N.TM_MATCH_ALL):
            if hs is None:
                out.append(BadArg("'#' before the last level"))
                continue
            keys = [self._key_of(h) for h in hs]
            if not opts:
                keys.sort(key=_key_order, reverse=True)
            out.append(self._reduce(keys, opts))
        return out

    def matches_filter(self, topic_filter, tab=None, opts=()):
        r = self.matches_filter_batch([topic_filter], opts)[0]
        if isinstance(r, BadArg):
            raise r
        return r

    def match(self, topic, tab=None):
        """match/2: the first key in ETS term order, or False."""
        r = self.matches(topic, None, ["return_first"])
        return r[0] if r else False

    def get_record(self, key, tab=None):
        return self._records.get(key)

    def stats(self):
        return self.eng.stats()

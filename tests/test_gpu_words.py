"""matches/3 with pre-split topics `[word()]` (emqx_trie_search.erl:182, topic_words/1
:369-370) through the C-ABI: tm_match_batch with TM_MATCH_TOPIC_WORDS.

Expected sets are computed here from the reference's definitions, per topic word list W:
  - every word-list key (wildcard filters and exact keys inserted as lists) whose words
    match W under emqx_topic:match/2's list clauses (emqx_topic.erl:90-101), a "+" or "#"
    word of W being a plain binary word (topic_words/1 checks nothing for a list);
  - the '$' rule of base_init/1 (emqx_trie_search.erl:160-163): a first word starting with
    '$' is never reached by a filter starting with '+' or '#';
  - keys given as binaries ({Binary, {ID}}) never: match_topics/4 compares the list itself
    with the keys (:380-389).
The walk restatement (oracle/) pins the same sets for topics without "+"/"#" words: the
binary topic's oracle result minus its binary keys.
"""
import numpy as np
import pytest

import oracle
from emqx_amd import _native as N
from emqx_amd import workloads
from oracle import emqx_topic as et

pytestmark = pytest.mark.gpu


def _filter_words(f: bytes):
    return ["+" if w == b"+" else "#" if w == b"#" else w for w in f.split(b"/")]


def _expected(keys, W):
    """keys: (filter bytes, id, is_list_key); W: list of byte words."""
    out = []
    for f, i, is_list in keys:
        if not is_list:
            continue
        fw = _filter_words(f)
        if W[0][:1] == b"$" and fw[0] in ("+", "#"):
            continue
        if et._match_words(list(W), fw):
            out.append(i)
    return sorted(out)


def test_word_list_topics_vs_reference_definitions():
    rng = np.random.default_rng(11)
    vocab = [b"a", b"b", b"c", b"", b"$SYS", b"+", b"#", b"dev7", b"x"]
    keys = []
    for i in range(1, 600):
        nl = int(rng.integers(1, 5))
        ws = [vocab[int(rng.integers(0, 5))] if rng.random() < 0.8 else b"+" for _ in range(nl)]
        ws = [b"a" if w in (b"+", b"#") and rng.random() < 0.3 else w for w in ws]
        if rng.random() < 0.25:
            ws[-1] = b"#"
        if rng.random() < 0.1:
            ws[0] = b"$SYS"
        f = b"/".join(ws)
        wild = b"+" in ws or b"#" in ws
        as_list = wild or rng.random() < 0.5  # exact filters: half inserted as word lists
        keys.append((f, i, as_list))
    eng = N.Engine(0)
    buf, off = N.pack_topics([k[0] for k in keys])
    ids = np.array([k[1] for k in keys], np.uint64)
    flags = np.array([N.TM_KEY_WORDS if k[2] else 0 for k in keys], np.uint32)
    eng.apply_packed(N.TM_OP_ADD, buf, off.astype(np.uint64), ids, flags)
    eng.commit()
    topics = [[vocab[int(rng.integers(0, len(vocab)))] for _ in range(int(rng.integers(1, 6)))] for _ in range(3000)]
    topics += [[b"a"], [b"+"], [b"#"], [b"$SYS", b"a"], [b""], [b"a", b"#"], [b"a", b"+", b"c"]]
    got = eng.match_words(topics)
    kid = {}
    for w, hs in zip(topics, got):
        ids_got = sorted(eng.key_info(h)[0] for h in hs)
        assert ids_got == _expected(keys, w), w
        kid[tuple(w)] = ids_got
    # COUNT / FIRST / UNIQUE on the same topics
    _, cnt, _, _ = eng.match_packed(*N.pack_topics([b"/".join(w) for w in topics]),
                                    N.TM_MATCH_COUNT | N.TM_MATCH_TOPIC_WORDS)
    assert [int(c) for c in cnt] == [len(kid[tuple(w)]) for w in topics]
    first = eng.match_words(topics, N.TM_MATCH_FIRST)
    for w, hs in zip(topics, first):
        assert len(hs) == (1 if kid[tuple(w)] else 0), w
        if hs:
            assert eng.key_info(hs[0])[0] in kid[tuple(w)]
    uniq = eng.match_words(topics, N.TM_MATCH_UNIQUE)
    for w, hs in zip(topics, uniq):
        assert sorted(eng.key_info(h)[0] for h in hs) == sorted(set(kid[tuple(w)])), w
    eng.close()


def test_word_list_topics_equal_the_walk_restatement_minus_binary_keys():
    """At config C scale 0.02 (word-list and binary exact keys mixed by id), topics without a
    "+"/"#" word: the oracle's walk of the binary topic, without the keys given as binaries."""
    w = workloads.generate("C", scale=0.02, n_topics=5000)
    flags = (w.f_id % 2).astype(np.uint32) * N.TM_KEY_WORDS  # half the exact keys as word lists
    eng = N.Engine(0)
    eng.apply_packed(N.TM_OP_ADD, w.f_bytes, w.f_off, w.f_id, flags)
    eng.commit()
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id, flags)
    eo, eids, est, esrc = ix.match(w.t_bytes, w.t_off, threads=8, with_src=True)
    fl = w.filters()
    is_bin = np.array([not (flags[k] or b"+" in fl[k].split(b"/") or b"#" in fl[k].split(b"/"))
                       for k in range(len(fl))])
    topics = [bytes(w.t_bytes[w.t_off[t]:w.t_off[t + 1]]).split(b"/") for t in range(w.n_topics)]
    got = eng.match_words(topics)
    for t in range(w.n_topics):
        if est[t]:
            continue  # a '+' / '#' level: badarg as a binary, a plain word as a list
        src = esrc[eo[t]:eo[t + 1]]
        exp = sorted(int(w.f_id[k]) for k in src if not is_bin[k])
        assert sorted(eng.key_ids(np.asarray(got[t], np.uint32)).tolist()) == exp, t
    eng.close()

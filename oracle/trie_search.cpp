// oracle/trie_search.cpp — TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).
//
// Nothing in the product (emqx_amd/) links, loads or calls this file.  Only tests/,
// __graft_entry__.smoke() and bench.py's cpu_baseline leg use it.
//
// Two CPU restatements of the reference's topic matching, both in plain C++:
//
// (1) brute force: emqx_topic:match/2 (apps/emqx/src/emqx_topic.erl:78-102) applied to
//     every key.  The semantic definition.
//
// (2) the indexed algorithm of emqx_trie_search (apps/emqx/src/emqx_trie_search.erl:192-389)
//     over an ordered key set with Erlang term order, as ETS ordered_set provides it
//     (apps/emqx/src/emqx_topic_index.erl:40-48,108-109):
//       - keys {Words, {ID}} for wildcard filters and word-list inserts, {Binary, {ID}}
//         for plain topics (make_key/2, :115-128);
//       - term order: lists < binaries; atoms '#' < '+' < every binary; binaries
//         bytewise, a prefix first; tuples by size first, so {P, {}} < {P, {ID}};
//       - next(K) = the smallest key > K, an O(log N) search like ets:next/2.
//     Words are ranked once so term comparisons are integer comparisons:
//     '#' -> 0, '+' -> 1, the k-th dictionary word (bytewise order) -> 2k+3, and a
//     topic word outside the dictionary -> 2*lower_bound+2 (between its neighbours).
//     This is the CPU baseline that bench.py times ("kind": "port").
//
// Third-party note: ETS itself (OTP 26.2.5.2, .tool-versions:1) is not under
// /root/reference; only its observable contract (ordered next/2) is restated.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

namespace {

constexpr uint32_t R_HASH = 0, R_PLUS = 1;

struct ListKey {
    uint64_t woff;  // into Index::wr
    uint32_t wlen;
    uint32_t src;   // input key index
    uint64_t id;
};
struct BinKey {
    uint64_t boff;  // into Index::bb
    uint32_t blen;
    uint32_t src;
    uint64_t id;
};

struct Index {
    std::vector<std::string> dict;                       // sorted distinct literal words
    std::unordered_map<std::string, uint32_t> dict_rank;  // word -> 2k+3
    std::vector<uint32_t> wr;                            // ranked words of list keys
    std::vector<ListKey> lk;                             // sorted in term order
    std::vector<uint8_t> bb;
    std::vector<BinKey> bk;                              // sorted in term order
    // brute force view: every key's tokens
    std::vector<std::vector<std::string>> fw;            // filter tokens per input key
    std::vector<uint8_t> fdollar_excl;                   // filter starts with '+' or '#' byte
    std::vector<uint64_t> fid;
    uint64_t nkeys = 0;
};

void split(const uint8_t *p, size_t n, std::vector<std::string> &out) {
    out.clear();
    size_t st = 0;
    for (size_t i = 0; i <= n; i++)
        if (i == n || p[i] == '/') {
            out.emplace_back((const char *)p + st, i - st);
            st = i + 1;
        }
}

int cmp_ranks(const uint32_t *a, uint32_t na, const uint32_t *b, uint32_t nb) {
    uint32_t n = std::min(na, nb);
    for (uint32_t i = 0; i < n; i++)
        if (a[i] != b[i]) return a[i] < b[i] ? -1 : 1;
    return na == nb ? 0 : (na < nb ? -1 : 1);
}

int cmp_bytes(const uint8_t *a, uint32_t na, const uint8_t *b, uint32_t nb) {
    int c = memcmp(a, b, std::min(na, nb));
    if (c) return c < 0 ? -1 : 1;
    return na == nb ? 0 : (na < nb ? -1 : 1);
}

// topic word -> rank (dictionary or in-between)
uint32_t topic_rank(const Index &ix, const std::string &w) {
    auto it = ix.dict_rank.find(w);
    if (it != ix.dict_rank.end()) return it->second;
    size_t k = std::lower_bound(ix.dict.begin(), ix.dict.end(), w) - ix.dict.begin();
    return (uint32_t)(2 * k + 2);
}

enum CmpKind { MATCH_FULL, MATCH_PREFIX, LOWER, SEEK };
struct CmpRes {
    CmpKind k;
    uint32_t pos, word;
};

// compare/3 (emqx_trie_search.erl:260-348) for a topic (not a filter) search.
CmpRes compare(const uint32_t *F, uint32_t FL, const uint32_t *W, uint32_t WL) {
    int last_plus = -1;
    for (uint32_t pos = 0;; pos++) {
        const bool fin = pos == FL, win = pos == WL;
        if (fin && win) return {MATCH_FULL, 0, 0};        // compare([], [], _)
        if (fin) return {MATCH_PREFIX, 0, 0};             // compare([], _Words, _)
        if (FL - pos == 1 && F[pos] == R_HASH) return {MATCH_FULL, 0, 0};  // compare(['#'], ...)
        if (F[pos] == R_PLUS && !win) {                   // compare(['+'|TF], [HW|TW], Pos)
            last_plus = (int)pos;
            continue;
        }
        if (!win && F[pos] == W[pos]) continue;           // compare([HW|TF], [HW|TW], Pos)
        if (win || F[pos] > W[pos]) {                     // lower (:325-340)
            if (last_plus >= 0) return {SEEK, (uint32_t)last_plus, W[last_plus]};
            return {LOWER, 0, 0};
        }
        return {SEEK, pos, W[pos]};                        // {Pos, HW} (:341-348)
    }
}

// compare/3 for a filter search (matches_filter/3, emqx_trie_search.erl:186-189): the
// topic-search clauses plus the two "Filter search" clauses (:291-300) -- a query '#' as
// the last word matches any remaining key words, a query '+' matches any one key word and
// passes the deeper result through unchanged (a `lower` there stays `lower`, so it is
// not a backtrack point).  Clause order as in the reference.
CmpRes compare_filter(const uint32_t *F, uint32_t FL, const uint32_t *W, uint32_t WL) {
    int last_plus = -1;
    for (uint32_t pos = 0;; pos++) {
        const bool fin = pos == FL, win = pos == WL;
        if (fin && win) return {MATCH_FULL, 0, 0};                          // compare([], [], _)
        if (fin) return {MATCH_PREFIX, 0, 0};                               // compare([], _Words, _)
        if (FL - pos == 1 && F[pos] == R_HASH) return {MATCH_FULL, 0, 0};   // compare(['#'], ...)
        if (!win && WL - pos == 1 && W[pos] == R_HASH) return {MATCH_FULL, 0, 0};  // compare(_, ['#'], _)
        if (!win && W[pos] == R_PLUS) continue;                             // compare([_|TF], ['+'|TW], Pos)
        if (F[pos] == R_PLUS && !win) {                                     // compare(['+'|TF], [HW|TW], Pos)
            last_plus = (int)pos;
            continue;
        }
        if (!win && F[pos] == W[pos]) continue;                             // compare([HW|TF], [HW|TW], Pos)
        if (win || F[pos] > W[pos]) {                                       // lower (:325-340)
            if (last_plus >= 0) return {SEEK, (uint32_t)last_plus, W[last_plus]};
            return {LOWER, 0, 0};
        }
        return {SEEK, pos, W[pos]};                                         // {Pos, HW} (:341-348)
    }
}

// ETS-like positions: [0, NL) list keys, [NL, NL+NB) binary keys, NL+NB = '$end_of_table'
struct Searcher {
    const Index &ix;
    std::vector<uint32_t> prefix;
    explicit Searcher(const Index &i) : ix(i) {}

    // next({Prefix, {}}) over list keys: first list key with words >= Prefix
    size_t next_base_list(const uint32_t *p, uint32_t n) const {
        size_t lo = 0, hi = ix.lk.size();
        while (lo < hi) {
            size_t mid = (lo + hi) / 2;
            const ListKey &k = ix.lk[mid];
            if (cmp_ranks(&ix.wr[k.woff], k.wlen, p, n) < 0) lo = mid + 1;
            else hi = mid;
        }
        return lo;  // == NL: continues into the binary keys
    }
    // next({Topic, {}}) over binary keys
    size_t next_base_bin(const uint8_t *t, uint32_t n) const {
        size_t lo = 0, hi = ix.bk.size();
        while (lo < hi) {
            size_t mid = (lo + hi) / 2;
            const BinKey &k = ix.bk[mid];
            if (cmp_bytes(&ix.bb[k.boff], k.blen, t, n) < 0) lo = mid + 1;
            else hi = mid;
        }
        return ix.lk.size() + lo;
    }

    // search/3 with opts [] (mode 0), [unique] (1), [return_first] (2); appends input
    // key indices to out in the order the reference's accumulator would hold them
    // reversed (we emit in walk order).
    void search(const uint8_t *topic, uint32_t tlen, const uint32_t *W, uint32_t WL, int mode,
                std::vector<uint32_t> &out) {
        const size_t NL = ix.lk.size(), END = NL + ix.bk.size();
        // base_init/1 (:160-163): '$' topics start at [W0], skipping root '+'/'#'
        size_t cur;
        if (tlen && topic[0] == '$') cur = next_base_list(W, 1);
        else cur = next_base_list(nullptr, 0);
        auto add = [&](uint32_t src) -> bool {
            out.push_back(src);
            return mode == 2;  // return_first: stop at the first hit
        };
        // search_new / search_up loop (:230-253)
        for (;;) {
            if (cur == END) return;
            if (cur >= NL) break;  // binary key: compare(NotFilter, ...) -> lower
            const ListKey &k = ix.lk[cur];
            CmpRes r = compare(&ix.wr[k.woff], k.wlen, W, WL);
            if (r.k == MATCH_FULL) {
                if (add(k.src)) return;
                cur++;
            } else if (r.k == MATCH_PREFIX) {
                cur++;
            } else if (r.k == LOWER) {
                break;
            } else {
                // seek/3 (:255-258): first Pos filter words + [SeekWord]
                prefix.assign(&ix.wr[k.woff], &ix.wr[k.woff] + r.pos);
                prefix.push_back(r.word);
                cur = next_base_list(prefix.data(), (uint32_t)prefix.size());
            }
        }
        // match_topics/4 (:381-389): exact binary keys
        for (;;) {
            if (cur == END) return;
            if (cur < NL) {  // a list key is < any binary: jump to {Topic, {}}
                cur = next_base_bin(topic, tlen);
                continue;
            }
            const BinKey &k = ix.bk[cur - NL];
            int c = cmp_bytes(&ix.bb[k.boff], k.blen, topic, tlen);
            if (c == 0) {
                if (add(k.src)) return;
                cur++;
            } else if (c < 0) {
                cur = next_base_bin(topic, tlen);
            } else {
                return;
            }
        }
    }
};

// matches_filter/3 (emqx_trie_search.erl:186-189,192-228 with topic_filter set): the
// same search_new/search_up loop over the list keys only -- a binary key compares
// `lower` and the filter search never runs match_topics/4.  Appends input key indices in
// walk order (the reference's accumulator holds them reversed).
void search_filter(const Index &ix, const uint8_t *q, uint32_t qlen, const uint32_t *W, uint32_t WL, int mode,
                   std::vector<uint32_t> &out, std::vector<uint32_t> &prefix, const Searcher &S) {
    const size_t NL = ix.lk.size();
    // base_init/1 (:160-163): a first word <<"$", _/bytes>> starts at [W0]
    size_t cur = (qlen && q[0] == '$') ? S.next_base_list(W, 1) : S.next_base_list(nullptr, 0);
    while (cur < NL) {
        const ListKey &k = ix.lk[cur];
        CmpRes r = compare_filter(&ix.wr[k.woff], k.wlen, W, WL);
        if (r.k == MATCH_FULL) {
            out.push_back(k.src);
            if (mode == 2) return;
            cur++;
        } else if (r.k == MATCH_PREFIX) {
            cur++;
        } else if (r.k == LOWER) {
            return;
        } else {
            prefix.assign(&ix.wr[k.woff], &ix.wr[k.woff] + r.pos);
            prefix.push_back(r.word);
            cur = S.next_base_list(prefix.data(), (uint32_t)prefix.size());
        }
    }
}

// emqx_topic:match/2 on token lists (emqx_topic.erl:78-102); tokens are bytes, '+'/'#'
// levels are wildcards in the filter only.
bool brute_match(const std::vector<std::string> &T, bool tdollar, const std::vector<std::string> &F,
                 bool fexcl) {
    if (tdollar && fexcl) return false;  // match(<<$$,_>>, <<$+,_>> | <<$#,_>>) -> false
    size_t i = 0;
    for (;; i++) {
        if (i == F.size()) return i == T.size();
        if (F[i] == "#" && i + 1 == F.size()) return true;  // match(_, ['#'])
        if (i == T.size()) return false;
        if (F[i] == "+") continue;
        if (F[i] != T[i]) return false;
    }
}

}  // namespace

extern "C" {

// Build the ordered key set.  Key i: bytes[off[i]..off[i+1]), id ids[i], flags[i]&1 =
// given as a word list.  Duplicate (key, id) pairs collapse (ETS set semantics).
void *ots_build(const uint8_t *bytes, const uint64_t *off, const uint64_t *ids, const uint32_t *flags, uint64_t n) {
    Index *ix = new Index();
    ix->nkeys = n;
    ix->fw.resize(n);
    ix->fdollar_excl.resize(n);
    ix->fid.assign(ids, ids + n);
    std::vector<std::string> tok;
    std::vector<char> is_list(n);
    // dictionary of literal words appearing in list keys
    std::vector<std::string> words;
    for (uint64_t i = 0; i < n; i++) {
        const uint8_t *p = bytes + off[i];
        size_t len = off[i + 1] - off[i];
        split(p, len, ix->fw[i]);
        ix->fdollar_excl[i] = len && (p[0] == '+' || p[0] == '#');
        bool wild = false;
        for (auto &w : ix->fw[i])
            if (w == "+" || w == "#") wild = true;
        is_list[i] = wild || (flags && (flags[i] & 1));
        if (is_list[i])
            for (auto &w : ix->fw[i])
                if (w != "+" && w != "#") words.push_back(w);
    }
    std::sort(words.begin(), words.end());
    words.erase(std::unique(words.begin(), words.end()), words.end());
    ix->dict = words;
    ix->dict_rank.reserve(words.size() * 2);
    for (size_t k = 0; k < words.size(); k++) ix->dict_rank[words[k]] = (uint32_t)(2 * k + 3);
    for (uint64_t i = 0; i < n; i++) {
        if (is_list[i]) {
            ListKey k{ix->wr.size(), (uint32_t)ix->fw[i].size(), (uint32_t)i, ids[i]};
            for (auto &w : ix->fw[i])
                ix->wr.push_back(w == "#" ? R_HASH : w == "+" ? R_PLUS : ix->dict_rank[w]);
            ix->lk.push_back(k);
        } else {
            BinKey k{ix->bb.size(), (uint32_t)(off[i + 1] - off[i]), (uint32_t)i, ids[i]};
            ix->bb.insert(ix->bb.end(), bytes + off[i], bytes + off[i + 1]);
            ix->bk.push_back(k);
        }
    }
    auto lcmp = [&](const ListKey &a, const ListKey &b) {
        int c = cmp_ranks(&ix->wr[a.woff], a.wlen, &ix->wr[b.woff], b.wlen);
        return c ? c < 0 : a.id < b.id;
    };
    auto leq = [&](const ListKey &a, const ListKey &b) {
        return cmp_ranks(&ix->wr[a.woff], a.wlen, &ix->wr[b.woff], b.wlen) == 0 && a.id == b.id;
    };
    std::sort(ix->lk.begin(), ix->lk.end(), lcmp);
    ix->lk.erase(std::unique(ix->lk.begin(), ix->lk.end(), leq), ix->lk.end());
    auto bcmp = [&](const BinKey &a, const BinKey &b) {
        int c = cmp_bytes(&ix->bb[a.boff], a.blen, &ix->bb[b.boff], b.blen);
        return c ? c < 0 : a.id < b.id;
    };
    auto beq = [&](const BinKey &a, const BinKey &b) {
        return cmp_bytes(&ix->bb[a.boff], a.blen, &ix->bb[b.boff], b.blen) == 0 && a.id == b.id;
    };
    std::sort(ix->bk.begin(), ix->bk.end(), bcmp);
    ix->bk.erase(std::unique(ix->bk.begin(), ix->bk.end(), beq), ix->bk.end());
    return ix;
}

void ots_free(void *h) { delete (Index *)h; }

uint64_t ots_size(void *h) {
    Index *ix = (Index *)h;
    return ix->lk.size() + ix->bk.size();
}

// Result buffers owned by a handle: per-topic counts + flattened ids.
struct Results {
    std::vector<uint32_t> cnt;
    std::vector<int32_t> status;
    std::vector<std::vector<uint64_t>> ids;   // sorted ids per topic
    std::vector<std::vector<uint32_t>> srcs;  // input key indices per topic, walk order
    std::vector<uint64_t> flat;
    std::vector<uint32_t> flat_src;
    std::vector<uint64_t> off;
};

static void to_words(const Index &ix, const uint8_t *t, uint32_t n, std::vector<std::string> &tok,
                     std::vector<uint32_t> &W, bool *badarg) {
    split(t, n, tok);
    W.resize(tok.size());
    *badarg = false;
    for (size_t i = 0; i < tok.size(); i++) {
        if (tok[i] == "+" || tok[i] == "#") *badarg = true;  // word/2 badarg (:374-375)
        W[i] = topic_rank(ix, tok[i]);
    }
}

// Match a batch with the trie-search restatement (algo 0), brute force (algo 1) or the
// filter search of matches_filter/3 (algo 2: queries are topic filters),
// mode 0 = [], 1 = [unique], 2 = return_first; nthreads workers.  Returns a results
// handle (per-topic ids sorted ascending) or, when `counts_only`, only fills
// cnt_out and returns nullptr.
void *ots_match(void *h, const uint8_t *bytes, const uint32_t *off, uint64_t n, int algo, int mode,
                int nthreads, int counts_only, uint32_t *cnt_out, uint64_t *checksum_out) {
    Index &ix = *(Index *)h;
    Results *R = counts_only ? nullptr : new Results();
    if (R) {
        R->cnt.resize(n);
        R->status.resize(n);
        R->ids.resize(n);
        R->srcs.resize(n);
    }
    std::atomic<uint64_t> next{0}, csum{0};
    if (nthreads < 1) nthreads = 1;
    auto worker = [&]() {
        Searcher S(ix);
        std::vector<std::string> tok;
        std::vector<uint32_t> W, out, prefix;
        uint64_t local = 0;
        for (;;) {
            uint64_t b = next.fetch_add(256);
            if (b >= n) break;
            uint64_t e = std::min<uint64_t>(b + 256, n);
            for (uint64_t i = b; i < e; i++) {
                const uint8_t *t = bytes + off[i];
                uint32_t tl = off[i + 1] - off[i];
                bool bad;
                out.clear();
                if (algo == 0) {
                    to_words(ix, t, tl, tok, W, &bad);
                    if (!bad) S.search(t, tl, W.data(), (uint32_t)W.size(), mode, out);
                } else if (algo == 2) {
                    // matches_filter/3: filter_words/1 (:356-366) -- '+'/'#' levels become
                    // the atoms, no badarg
                    split(t, tl, tok);
                    W.resize(tok.size());
                    for (size_t j = 0; j < tok.size(); j++)
                        W[j] = tok[j] == "#" ? R_HASH : tok[j] == "+" ? R_PLUS : topic_rank(ix, tok[j]);
                    // a '#' before the last level: the reference's walk does not terminate
                    // (a '+' key backtracks to seek word '#', which sorts below the key), so
                    // such a query is refused with the badarg status instead
                    bad = false;
                    for (size_t j = 0; j + 1 < W.size(); j++)
                        if (W[j] == R_HASH) bad = true;
                    if (!bad) search_filter(ix, t, tl, W.data(), (uint32_t)W.size(), mode, out, prefix, S);
                } else {
                    split(t, tl, tok);
                    bad = false;
                    for (auto &w : tok)
                        if (w == "+" || w == "#") bad = true;
                    bool td = tl && t[0] == '$';
                    if (!bad)
                        for (uint64_t k = 0; k < ix.nkeys; k++)
                            if (brute_match(tok, td, ix.fw[k], ix.fdollar_excl[k])) out.push_back((uint32_t)k);
                }
                uint64_t c = out.size();
                for (uint32_t s : out) local += ix.fid[s] * 0x9E3779B97F4A7C15ull + i;
                if (cnt_out) cnt_out[i] = (uint32_t)c;
                if (R) {
                    R->status[i] = bad ? 1 : 0;
                    std::vector<uint64_t> &v = R->ids[i];
                    for (uint32_t s : out) v.push_back(ix.fid[s]);
                    R->srcs[i] = out;
                    std::sort(v.begin(), v.end());
                    if (mode == 1) v.erase(std::unique(v.begin(), v.end()), v.end());  // [unique]
                    R->cnt[i] = (uint32_t)v.size();
                }
            }
        }
        csum.fetch_add(local);
    };
    std::vector<std::thread> th;
    for (int k = 1; k < nthreads; k++) th.emplace_back(worker);
    worker();
    for (auto &t : th) t.join();
    if (checksum_out) *checksum_out = csum.load();
    if (R) {
        R->off.resize(n + 1);
        R->off[0] = 0;
        for (uint64_t i = 0; i < n; i++) R->off[i + 1] = R->off[i] + R->ids[i].size();
        R->flat.reserve(R->off[n]);
        for (auto &v : R->ids) R->flat.insert(R->flat.end(), v.begin(), v.end());
        R->ids.clear();
        R->ids.shrink_to_fit();
        // walk-order sources (same per-topic counts except under [unique])
        for (auto &v : R->srcs) R->flat_src.insert(R->flat_src.end(), v.begin(), v.end());
        R->srcs.clear();
        R->srcs.shrink_to_fit();
    }
    return R;
}

const uint64_t *ots_res_off(void *r) { return ((Results *)r)->off.data(); }
const uint64_t *ots_res_ids(void *r) { return ((Results *)r)->flat.data(); }
const int32_t *ots_res_status(void *r) { return ((Results *)r)->status.data(); }
uint64_t ots_res_nsrc(void *r) { return ((Results *)r)->flat_src.size(); }
const uint32_t *ots_res_src(void *r) { return ((Results *)r)->flat_src.data(); }
void ots_res_free(void *r) { delete (Results *)r; }

}  // extern "C"

// ---------------------------------------------------------------------------
// emqx_topic:intersection/2 (apps/emqx/src/emqx_topic.erl:111-151) + join/1 (:310-322),
// restated over byte words ('+' / '#' are the wildcard levels, every other level -- the
// empty one included -- a literal compared bytewise).  The C++ CPU baseline of the
// intersection leg (bench.py) and its parity checker over whole batches.
// Per pair: out_len[i] = result length, -1 = false, -2 = error('topic_invalid_#') from
// join/1; the result bytes at out + a_off[i] + b_off[i] (room: both inputs' lengths + 1).
namespace {
struct W {
    const uint8_t *p;
    uint32_t n;
    bool plus() const { return n == 1 && p[0] == '+'; }
    bool hash() const { return n == 1 && p[0] == '#'; }
    bool wild() const { return plus() || hash(); }
    bool eq(const W &o) const { return n == o.n && std::memcmp(p, o.p, n) == 0; }
};
void words_of(const uint8_t *p, uint32_t n, std::vector<W> &out) {
    out.clear();
    uint32_t st = 0;
    for (uint32_t i = 0; i <= n; i++)
        if (i == n || p[i] == '/') {
            out.push_back(W{p + st, i - st});
            st = i + 1;
        }
}
const W PLUS_W{(const uint8_t *)"+", 1};
// intersect/2 (:128-151): false, or the intersection's words
bool intersect_words(const std::vector<W> &a, const std::vector<W> &b, std::vector<W> &r) {
    r.clear();
    size_t i = 0, j = 0;
    for (;;) {
        const size_t ra = a.size() - i, rb = b.size() - j;
        if (rb == 1 && b[j].hash()) {  // intersect(Words, ['#']) -> Words
            r.insert(r.end(), a.begin() + i, a.end());
            return true;
        }
        if (ra == 1 && a[i].hash()) {  // intersect(['#'], Words) -> Words
            r.insert(r.end(), b.begin() + j, b.end());
            return true;
        }
        if (ra == 1 && rb == 1 && b[j].plus()) {  // intersect([W], ['+']) -> [W]
            r.push_back(a[i]);
            return true;
        }
        if (ra == 1 && rb == 1 && a[i].plus()) {  // intersect(['+'], [W]) -> [W]
            r.push_back(b[j]);
            return true;
        }
        if (ra && rb) {
            const W &x = a[i], &y = b[j];
            if (x.wild() && y.wild()) r.push_back(x.eq(y) ? x : PLUS_W);
            else if (x.eq(y)) r.push_back(x);
            else if (x.wild()) r.push_back(y);
            else if (y.wild()) r.push_back(x);
            else return false;
            i++;
            j++;
            continue;
        }
        return ra == 0 && rb == 0;  // intersect([], []) -> []; anything else -> false
    }
}
bool dollar_first(const std::vector<W> &w) { return w[0].n && w[0].p[0] == '$' && !w[0].wild(); }
}  // namespace

extern "C" void ots_intersect(const uint8_t *a_buf, const uint32_t *a_off, const uint8_t *b_buf, const uint32_t *b_off,
                              uint64_t n, int nthreads, uint8_t *out, int32_t *out_len) {
    std::atomic<uint64_t> next{0};
    if (nthreads < 1) nthreads = 1;
    auto worker = [&]() {
        std::vector<W> a, b, r;
        for (;;) {
            const uint64_t lo = next.fetch_add(4096);
            if (lo >= n) break;
            const uint64_t hi = std::min<uint64_t>(lo + 4096, n);
            for (uint64_t i = lo; i < hi; i++) {
                words_of(a_buf + a_off[i], a_off[i + 1] - a_off[i], a);
                words_of(b_buf + b_off[i], b_off[i + 1] - b_off[i], b);
                // '$'-topics never intersect a filter whose first level is a wildcard (:113-118)
                if ((dollar_first(a) && b[0].wild()) || (dollar_first(b) && a[0].wild()) ||
                    !intersect_words(a, b, r)) {
                    out_len[i] = -1;
                    continue;
                }
                bool bad = false;  // join/1: '#' anywhere but last
                for (size_t k = 0; k + 1 < r.size(); k++)
                    if (r[k].hash()) bad = true;
                if (bad) {
                    out_len[i] = -2;
                    continue;
                }
                uint8_t *o = out + (uint64_t)a_off[i] + b_off[i];
                uint32_t len = 0;
                for (size_t k = 0; k < r.size(); k++) {
                    if (k) o[len++] = '/';
                    std::memcpy(o + len, r[k].p, r[k].n);
                    len += r[k].n;
                }
                out_len[i] = (int32_t)len;
            }
        }
    };
    std::vector<std::thread> th;
    for (int k = 1; k < nthreads; k++) th.emplace_back(worker);
    worker();
    for (auto &t : th) t.join();
}

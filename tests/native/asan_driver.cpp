// tests/native/asan_driver.cpp — the host side of libemqx_tm under AddressSanitizer and
// UndefinedBehaviorSanitizer (sanitizers on the host C++ library; the GPU
// code is built normally — device sanitizers are not available on this pool).
//
// Built by tests/native/Makefile with hipcc, `-Xarch_host -fsanitize=...` so only host
// code is instrumented.  Exercises every C-ABI entry point through a seeded churn of
// adds/deletes (incl. invalid and $-filters, word-list keys, re-adds inside one epoch),
// matches in every mode, key introspection, result shaping and the shard merge, and
// checks the modes against each other: COUNT == |ALL|, FIRST in ALL, UNIQUE subset of ALL.
// Then the batching aggregator (include/emqx_tm_batcher.h): 8 publisher threads with
// blocking publishes while the main thread commits epochs through the batcher.
#include <algorithm>
#include <atomic>
#include <thread>
#include <cstdio>
#include <unistd.h>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>
#include <string>
#include <vector>

#include "../../include/emqx_tm.h"
#include "../../include/emqx_tm_batcher.h"

#define CHECK(c)                                                           \
    do {                                                                   \
        if (!(c)) {                                                        \
            fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
            exit(1);                                                       \
        }                                                                  \
    } while (0)

static std::string rand_filter(std::mt19937_64 &r) {
    static const char *W[] = {"a", "b", "c", "", "foo", "$SYS", "x1", "long-level-word-123", "+", "+", "#"};
    int n = 1 + r() % 5;
    std::string f;
    for (int i = 0; i < n; i++) {
        if (i) f += '/';
        f += W[r() % 11];
    }
    return f;
}

static std::string rand_topic(std::mt19937_64 &r) {
    static const char *W[] = {"a", "b", "c", "", "foo", "$SYS", "x1", "long-level-word-123"};
    int n = 1 + r() % 6;
    std::string t;
    for (int i = 0; i < n; i++) {
        if (i) t += '/';
        t += W[r() % 8];
    }
    return t;
}

int main() {
    tm_config cfg;
    memset(&cfg, 0, sizeof cfg);
    tm_engine *eng = nullptr;
    CHECK(tm_create(&cfg, &eng) == TM_OK);
    std::mt19937_64 r(12345);
    struct Key {
        std::string f;
        uint64_t id;
        uint32_t flags;
    };
    std::vector<Key> live;
    uint64_t next_id = 1;
    for (int epoch = 0; epoch < 30; epoch++) {
        std::vector<std::string> keep;  // filter storage for the ops of this epoch
        std::vector<tm_op> ops;
        keep.reserve(4096);
        for (int i = 0; i < 200; i++) {
            tm_op o;
            memset(&o, 0, sizeof o);
            if (!live.empty() && r() % 3 == 0) {
                size_t k = r() % live.size();
                keep.push_back(live[k].f);
                o.op = TM_OP_DEL;
                o.id = live[k].id;
                o.flags = live[k].flags;  // a word-list key is deleted as a word list
                live[k] = live.back();
                live.pop_back();
            } else {
                keep.push_back(rand_filter(r));
                o.op = TM_OP_ADD;
                o.id = next_id++;
                o.flags = (r() % 7 == 0) ? TM_KEY_WORDS : 0;
                live.push_back({keep.back(), o.id, o.flags});
            }
            o.filter = (const uint8_t *)keep.back().data();
            o.filter_len = (uint32_t)keep.back().size();
            ops.push_back(o);
        }
        // re-add then delete inside the same epoch: last op wins
        keep.push_back("a/+/#");
        tm_op a;
        memset(&a, 0, sizeof a);
        a.op = TM_OP_ADD;
        a.filter = (const uint8_t *)keep.back().data();
        a.filter_len = (uint32_t)keep.back().size();
        a.id = 999999;
        ops.push_back(a);
        a.op = TM_OP_DEL;
        ops.push_back(a);
        CHECK(tm_apply(eng, ops.data(), ops.size()) == TM_OK);
        uint64_t ep = 0;
        CHECK(tm_commit_epoch(eng, &ep) == TM_OK);

        std::string bytes;
        std::vector<uint32_t> off{0};
        for (int i = 0; i < 300; i++) {
            bytes += (i % 50 == 0) ? std::string("a/+/b") : rand_topic(r);
            off.push_back((uint32_t)bytes.size());
        }
        bytes += std::string(16, '\0');
        const uint32_t n = (uint32_t)off.size() - 1;
        tm_result all, res;
        CHECK(tm_match_batch(eng, (const uint8_t *)bytes.data(), off.data(), n, TM_MATCH_ALL, &all) == TM_OK);
        std::vector<uint32_t> acnt(all.cnt, all.cnt + n), aoff(all.off, all.off + n);
        std::vector<uint32_t> akeys(all.keys, all.keys + all.total);
        std::vector<int32_t> ast(all.status, all.status + n);
        CHECK(tm_match_batch(eng, (const uint8_t *)bytes.data(), off.data(), n, TM_MATCH_COUNT, &res) == TM_OK);
        for (uint32_t i = 0; i < n; i++) CHECK(res.cnt[i] == acnt[i] && res.status[i] == ast[i]);
        CHECK(tm_match_batch(eng, (const uint8_t *)bytes.data(), off.data(), n, TM_MATCH_FIRST, &res) == TM_OK);
        for (uint32_t i = 0; i < n; i++) {
            CHECK(res.cnt[i] == (acnt[i] ? 1u : 0u));
            if (res.cnt[i]) {
                bool found = false;
                for (uint32_t k = 0; k < acnt[i]; k++) found |= akeys[aoff[i] + k] == res.keys[res.off[i]];
                CHECK(found);
            }
        }
        CHECK(tm_match_batch(eng, (const uint8_t *)bytes.data(), off.data(), n, TM_MATCH_UNIQUE, &res) == TM_OK);
        for (uint32_t i = 0; i < n; i++) {
            CHECK(res.cnt[i] <= acnt[i]);
            CHECK(acnt[i] == 0 || res.cnt[i] >= 1);
            // one key per id, and every id of the full set is there
            std::vector<uint64_t> uid(res.cnt[i]), aid(acnt[i]);
            CHECK(tm_key_ids(eng, res.keys + res.off[i], res.cnt[i], uid.data()) == TM_OK);
            CHECK(tm_key_ids(eng, akeys.data() + aoff[i], acnt[i], aid.data()) == TM_OK);
            std::sort(uid.begin(), uid.end());
            std::sort(aid.begin(), aid.end());
            aid.erase(std::unique(aid.begin(), aid.end()), aid.end());
            CHECK(uid == aid);
        }
        CHECK(tm_match_batch(eng, (const uint8_t *)bytes.data(), off.data(), n, TM_MATCH_AGGRE, &res) == TM_OK);
        for (uint32_t i = 0; i < n; i++) {
            CHECK(res.cnt[i] <= acnt[i]);
            for (uint32_t k = 0; k < res.cnt[i]; k++) {
                bool found = false;
                for (uint32_t j = 0; j < acnt[i]; j++) found |= akeys[aoff[i] + j] == res.keys[res.off[i] + k];
                CHECK(found);
            }
        }
        // matches_filter/3 on filters made from the topics (last level -> '#', and a few
        // refused ones with '#' before the last level); modes checked against ALL
        {
            std::string fb;
            std::vector<uint32_t> fo{0};
            for (uint32_t i = 0; i < n; i++) {
                std::string t = bytes.substr(off[i], off[i + 1] - off[i]);
                if (i % 3 == 1) t = t.substr(0, t.rfind('/') == std::string::npos ? 0 : t.rfind('/') + 1) + "#";
                if (i % 97 == 5) t = "#/" + t;
                fb += t;
                fo.push_back((uint32_t)fb.size());
            }
            tm_result fa, fr;
            CHECK(tm_match_filter_batch(eng, (const uint8_t *)fb.data(), fo.data(), n, TM_MATCH_ALL, &fa) == TM_OK);
            std::vector<uint32_t> fcnt(fa.cnt, fa.cnt + n), foff(fa.off, fa.off + n), fkeys(fa.keys, fa.keys + fa.total);
            for (uint32_t i = 0; i < n; i++) CHECK((fa.status[i] == TM_BADARG) == (i % 97 == 5) && foff[i] + fcnt[i] <= fa.total);
            CHECK(tm_match_filter_batch(eng, (const uint8_t *)fb.data(), fo.data(), n, TM_MATCH_FIRST, &fr) == TM_OK);
            for (uint32_t i = 0; i < n; i++)
                CHECK(fr.cnt[i] == (fcnt[i] ? 1u : 0u) && (!fr.cnt[i] || fr.keys[fr.off[i]] == fkeys[foff[i]]));
            CHECK(tm_match_filter_batch(eng, (const uint8_t *)fb.data(), fo.data(), n, TM_MATCH_UNIQUE, &fr) == TM_OK);
            for (uint32_t i = 0; i < n; i++) {
                std::vector<uint64_t> uid(fr.cnt[i]), aid(fcnt[i]);
                CHECK(tm_key_ids(eng, fr.keys + fr.off[i], fr.cnt[i], uid.data()) == TM_OK);
                CHECK(tm_key_ids(eng, fkeys.data() + foff[i], fcnt[i], aid.data()) == TM_OK);
                std::sort(aid.begin(), aid.end());
                aid.erase(std::unique(aid.begin(), aid.end()), aid.end());
                CHECK(uid == aid);  // listed by id
            }
            // intersection/2 of neighbouring filters
            tm_intersect_result ir;
            CHECK(tm_intersect_batch(eng, (const uint8_t *)fb.data(), fo.data(), (const uint8_t *)fb.data(),
                                     fo.data() + 1, n - 1, &ir) == TM_OK);
            for (uint32_t i = 0; i + 1 < n; i++) {
                CHECK(ir.len[i] >= TM_INTERSECT_BADHASH);
                CHECK(ir.len[i] < 0 || (uint64_t)ir.len[i] <= (uint64_t)(fo[i + 1] - fo[i]) + (fo[i + 2] - fo[i + 1]));
            }
        }
        // introspection of every matched key
        for (uint32_t k : akeys) {
            uint64_t id = 0;
            uint32_t fl = 0, len = 0;
            char buf[256];
            CHECK(tm_key_info(eng, k, &id, &fl, (uint8_t *)buf, sizeof buf, &len) == TM_OK);
            CHECK(len < sizeof buf);
        }
        std::vector<uint64_t> ids(akeys.size() + 1);
        CHECK(tm_key_ids(eng, akeys.data(), akeys.size(), ids.data()) == TM_OK);
        tm_stats_t st;
        CHECK(tm_stats(eng, &st) == TM_OK);
        if (st.n_keys != live.size()) {
            fprintf(stderr, "epoch %d: n_keys %llu vs %zu\n", epoch, (unsigned long long)st.n_keys, live.size());
            exit(1);
        }
        CHECK(st.epoch == ep);
    }
    // host shard merge
    {
        const uint32_t G = 3, n = 5;
        uint32_t counts[G * n];
        std::vector<uint64_t> ids(G * 16, 0);
        for (uint32_t i = 0; i < G * n; i++) counts[i] = i % 3;
        uint32_t outoff[n + 1];
        std::vector<uint64_t> outids(64);
        CHECK(tm_merge_shards(G, n, counts, ids.data(), 16, outoff, outids.data(), outids.size()) == TM_OK);
        CHECK(tm_merge_shards(G, n, counts, ids.data(), 16, outoff, outids.data(), 1) == TM_ENOMEM);
    }
    // batching aggregator: publishers race a commit that only ADDS keys under id 1<<40, so
    // every publish must return at least its ids from the epoch before (tm_match_batch) and
    // nothing outside the epoch after
    {
        std::vector<std::string> topics;
        for (int i = 0; i < 64; i++) topics.push_back(rand_topic(r));
        std::vector<uint8_t> tb;
        std::vector<uint32_t> to{0};
        for (auto &t : topics) {
            tb.insert(tb.end(), t.begin(), t.end());
            to.push_back((uint32_t)tb.size());
        }
        auto ids_of = [&](std::vector<std::multiset<uint64_t>> &out) {
            tm_result res;
            CHECK(tm_match_batch(eng, tb.data(), to.data(), (uint32_t)topics.size(), TM_MATCH_ALL, &res) == TM_OK);
            out.assign(topics.size(), {});
            for (size_t i = 0; i < topics.size(); i++) {
                std::vector<uint64_t> v(res.cnt[i] + 1);
                CHECK(tm_key_ids(eng, res.keys + res.off[i], res.cnt[i], v.data()) == TM_OK);
                out[i].insert(v.begin(), v.begin() + res.cnt[i]);
            }
        };
        std::vector<std::multiset<uint64_t>> before, after;
        ids_of(before);
        tm_batcher_config bc{16, 300, TM_MATCH_ALL, 0};
        tm_batcher *b = nullptr;
        CHECK(tm_batcher_create(eng, &bc, &b) == TM_OK);
        std::atomic<int> bad{0};
        std::vector<std::thread> th;
        for (int p = 0; p < 8; p++)
            th.emplace_back([&, p] {
                uint64_t ids[4096];
                for (int it = 0; it < 200; it++) {
                    const size_t i = (p * 131 + it * 7) % topics.size();
                    uint32_t n = 0;
                    int32_t st = 0;
                    if (tm_batcher_match(b, (const uint8_t *)topics[i].data(), (uint32_t)topics[i].size(), ids, 4096,
                                         &n, &st) != TM_OK || st != TM_TOPIC_OK || n > 4096) {
                        bad++;
                        continue;
                    }
                    std::multiset<uint64_t> got(ids, ids + n), old;
                    for (uint64_t x : got)
                        if (x < (1ull << 40)) old.insert(x);
                    if (old != before[i]) bad++;
                }
            });
        std::vector<tm_op> add;
        const char *nf[] = {"#", "a/#", "+/+", "a/b"};
        for (int k = 0; k < 4; k++) add.push_back(tm_op{TM_OP_ADD, 0, (const uint8_t *)nf[k], (uint32_t)strlen(nf[k]), 0,
                                                         (1ull << 40) + k});
        CHECK(tm_batcher_apply(b, add.data(), add.size()) == TM_OK);
        uint64_t ep2 = 0;
        CHECK(tm_batcher_commit(b, &ep2) == TM_OK);
        for (auto &t : th) t.join();
        CHECK(bad.load() == 0);
        tm_batcher_stats bs;
        CHECK(tm_batcher_stats_get(b, &bs) == TM_OK);
        CHECK(bs.publishes == 8 * 200 && bs.max_batch_seen <= 16 && bs.batches < bs.publishes);
        uint32_t n = 0;
        int32_t st = 0;
        CHECK(tm_batcher_match(b, (const uint8_t *)"a/+", 3, nullptr, 0, &n, &st) == TM_OK && st == TM_BADARG);
        tm_batcher_destroy(b);
        ids_of(after);
        for (size_t i = 0; i < topics.size(); i++) CHECK(after[i].size() >= before[i].size());
    }
    // big epochs (round 4): thousands of ops over thousands of distinct nodes, so every
    // parallel phase of a commit runs on the engine's helper threads under the sanitizer
    // (resolve, list builds, list placement, the upload's gathers; a full rebuild's too).
    // Each exact filter's own topic must match its key (exactly once while it is live).
    {
        std::vector<std::string> bigf;
        std::vector<uint64_t> bigid;
        std::vector<char> alive;
        uint64_t nid = 1ull << 41;
        for (int ep = 0; ep < 5; ep++) {
            std::vector<tm_op> ops;
            const size_t base = bigf.size();
            for (int i = 0; i < 6000; i++) {
                char fb[64];
                snprintf(fb, sizeof fb, "big/%d/n%zu/%s", i % 700, base + i, (i % 5 == 0) ? "+" : "x");
                bigf.push_back(fb);
                bigid.push_back(nid++);
                alive.push_back(1);
            }
            for (size_t k = 0; k < bigf.size(); k++) {  // adds of this epoch, and deletes of earlier ones
                if (k >= base) {
                    ops.push_back(tm_op{TM_OP_ADD, 0, (const uint8_t *)bigf[k].data(), (uint32_t)bigf[k].size(), 0, bigid[k]});
                } else if (alive[k] && (k * 2654435761u + ep) % 3 == 0) {
                    ops.push_back(tm_op{TM_OP_DEL, 0, (const uint8_t *)bigf[k].data(), (uint32_t)bigf[k].size(), 0, bigid[k]});
                    alive[k] = 0;
                }
            }
            CHECK(tm_apply(eng, ops.data(), ops.size()) == TM_OK);
            uint64_t ep3 = 0;
            CHECK(tm_commit_epoch(eng, &ep3) == TM_OK);
            std::string tb;
            std::vector<uint32_t> to{0};
            std::vector<size_t> which;
            for (size_t k = 0; k < bigf.size(); k += 7) {
                if (bigf[k].back() == '+') continue;
                tb += bigf[k];
                to.push_back((uint32_t)tb.size());
                which.push_back(k);
            }
            tm_result res;
            CHECK(tm_match_batch(eng, (const uint8_t *)tb.data(), to.data(), (uint32_t)which.size(), TM_MATCH_ALL, &res) ==
                  TM_OK);
            for (size_t i = 0; i < which.size(); i++) {
                std::vector<uint64_t> v(res.cnt[i] + 1);
                CHECK(tm_key_ids(eng, res.keys + res.off[i], res.cnt[i], v.data()) == TM_OK);
                const size_t own = std::count(v.begin(), v.begin() + res.cnt[i], bigid[which[i]]);
                CHECK(own == (alive[which[i]] ? 1u : 0u));
            }
        }
    }
    // bad arguments
    CHECK(tm_apply(eng, nullptr, 1) == TM_EINVAL);
    CHECK(tm_match_batch(eng, nullptr, nullptr, 0, 7, nullptr) == TM_EINVAL);
    tm_destroy(eng);
    printf("asan driver ok\n");
    fflush(stdout);
    // every engine and batcher is destroyed above (their frees ran under ASan); skip the HIP
    // runtime's own static teardown, where ASan's device-allocator quarantine can recycle a
    // chunk after the device runtime unloaded (a CHECK inside ASan, not a finding in this code)
    _exit(0);
}

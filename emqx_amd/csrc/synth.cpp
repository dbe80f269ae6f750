// synth.cpp — seeded synthetic route/topic sets for the BASELINE.json configs
// (A–E).  Workload generation only: not part of the matching path, built into
// its own library (libemqx_synth.so).
//
// Shape follows the reference's own generators:
//   * levels are hex words of width floor(1 + log2(V)/4) drawn from a per-level
//     vocabulary of V words, or one of the fixed words foo/bar/baz/xyzzy
//     (topic_level_t / topic_level_fixed_t, apps/emqx/test/emqx_topic_index_SUITE.erl:381-398);
//   * filters are made from a source topic by keeping levels, replacing levels with
//     '+', or cutting with '#' (mk_topic_filter, :410-419);
//   * $SYS topics look like "$SYS/brokers/<node>/<...>" (emqx_topic:systop/1,
//     apps/emqx/src/emqx_topic.erl:294-298);
//   * $share/G/F subscriptions become extra route keys on F with a different dest
//     (apps/emqx/src/emqx_shared_sub.erl:450): modelled as extra ids on one filter.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

namespace {

struct Rng {
    uint64_t s;
    explicit Rng(uint64_t seed) : s(seed) {}
    uint64_t next() {
        uint64_t z = (s += 0x9e3779b97f4a7c15ull);
        z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
        z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
        return z ^ (z >> 31);
    }
    double uni() { return (next() >> 11) * (1.0 / 9007199254740992.0); }
    uint32_t below(uint32_t n) { return n ? (uint32_t)((next() >> 32) * (uint64_t)n >> 32) : 0; }
};

// Zipf(s) over [0, n) by inverse CDF on a precomputed table (n small) or the
// continuous approximation (n large).
struct Zipf {
    uint32_t n = 1;
    double s = 0;
    std::vector<double> cdf;
    void init(uint32_t n_, double s_) {
        n = n_;
        s = s_;
        cdf.clear();
        if (s <= 0 || n > (1u << 16)) return;
        cdf.resize(n);
        double acc = 0;
        for (uint32_t i = 0; i < n; i++) {
            acc += 1.0 / std::pow((double)(i + 1), s);
            cdf[i] = acc;
        }
        for (auto &c : cdf) c /= acc;
    }
    uint32_t draw(Rng &r) const {
        if (s <= 0) return r.below(n);
        double u = r.uni();
        if (!cdf.empty()) {
            uint32_t lo = 0, hi = n - 1;
            while (lo < hi) {
                uint32_t mid = (lo + hi) / 2;
                if (cdf[mid] < u) lo = mid + 1;
                else hi = mid;
            }
            return lo;
        }
        // continuous approximation for large n (s != 1)
        double a = 1.0 - s;
        double x = std::abs(a) < 1e-9 ? std::exp(u * std::log((double)n)) : std::pow(u * (std::pow((double)n, a) - 1) + 1, 1.0 / a);
        uint32_t k = (uint32_t)x;
        return k >= 1 ? (k - 1 < n ? k - 1 : n - 1) : 0;
    }
};

}  // namespace

extern "C" {

typedef struct synth_params {
    uint64_t seed;
    uint64_t n_filters;     // distinct filter strings before extra ids
    uint64_t n_topics;
    uint32_t min_levels, max_levels;
    uint32_t vocab[16];     // per-level vocabulary (levels >= 16 use vocab[15])
    double zipf_s;          // word skew (0 = uniform)
    double p_fixed;         // level is one of foo/bar/baz/xyzzy
    double p_plus;          // filter gets '+' levels
    double p_plus_level;    // per-level chance of '+' in such a filter
    double p_hash;          // filter ends with '#'
    double hash_geo;        // '#' cut depth ~ min_hash_depth + Geometric(hash_geo)
    uint32_t min_hash_depth;
    uint32_t plus_hash_excl;  // 1: '#' filters never get '+' levels
    double p_topic_hit;     // topic derived from a random filter's source topic
    double p_sys;           // topic is a $SYS topic
    double p_sys_filter;    // filter is a $SYS filter
    double p_multi;         // a wildcard filter carries extra ids ($share groups g1..gK)
    uint32_t multi_max;     // extra ids ~ uniform [1, multi_max]
    uint32_t n_hot;         // hot '#' filters: many subscribers (ids) on one filter
    uint32_t hot_ids_min, hot_ids_max;  // ids per hot filter ~ log-uniform in [min, max]
    uint32_t hot_depth_min, hot_depth_max;
    double p_topic_hot;     // topic drawn under a random hot filter's prefix
    double hash_w[16];      // if any > 0: '#' cut depth d drawn with weight hash_w[d]
    uint32_t shard_count;   // > 1: emit only the route keys of shard `shard_index`
    uint32_t shard_index;   //      (shard_of(id) = splitmix64 finaliser(id) % shard_count)
} synth_params;

typedef struct synth_out {
    uint64_t n_keys;         // route keys (filter, id)
    uint8_t *f_bytes;
    uint64_t *f_off;         // n_keys + 1
    uint64_t *f_id;          // n_keys
    uint64_t n_topics;
    uint8_t *t_bytes;
    uint32_t *t_off;         // n_topics + 1 (batch offsets)
    uint64_t f_bytes_len, t_bytes_len;
} synth_out;

static void put_word(std::string &s, Rng &r, const synth_params &p, const std::vector<Zipf> &z, uint32_t level) {
    static const char *fixed[4] = {"foo", "bar", "baz", "xyzzy"};
    if (p.p_fixed > 0 && r.uni() < p.p_fixed) {
        s += fixed[r.below(4)];
        return;
    }
    uint32_t li = level < 16 ? level : 15;
    uint32_t V = p.vocab[li] ? p.vocab[li] : 16;
    uint32_t k = z[li].draw(r) + 1;
    int width = (int)std::floor(1 + std::log2((double)V) / 4);
    char buf[32];
    snprintf(buf, sizeof buf, "%0*X", width, k);
    s += buf;
}

static void gen_topic(std::vector<std::string> &lv, Rng &r, const synth_params &p, const std::vector<Zipf> &z) {
    uint32_t nl = p.min_levels + r.below(p.max_levels - p.min_levels + 1);
    lv.resize(nl);
    for (uint32_t i = 0; i < nl; i++) {
        lv[i].clear();
        put_word(lv[i], r, p, z, i);
    }
}

static std::string joinv(const std::vector<std::string> &lv, size_t n) {
    std::string s;
    for (size_t i = 0; i < n; i++) {
        if (i) s += '/';
        s += lv[i];
    }
    return s;
}

// The filter-sharded mode's key placement (emqx_amd/shard.py shard_of).
static uint64_t shard_mix(uint64_t x) {
    x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
    x ^= x >> 27; x *= 0x94d049bb133111ebull;
    return x ^ (x >> 31);
}

int synth_generate(const synth_params *pp, synth_out **out) {
    if (!pp || !out || pp->max_levels < pp->min_levels || pp->min_levels == 0) return -1;
    const synth_params &p = *pp;
    Rng r(p.seed);
    std::vector<Zipf> z(16);
    for (int i = 0; i < 16; i++) z[i].init(p.vocab[i] ? p.vocab[i] : 16, p.zipf_s);
    double wsum = 0;
    for (int i = 0; i < 16; i++) wsum += p.hash_w[i];

    std::vector<uint8_t> fb;
    std::vector<uint64_t> foff{0}, fid;
    std::vector<uint64_t> src_seed;  // rng seed of each filter's source topic
    const uint64_t kept = p.n_filters / (p.shard_count > 1 ? p.shard_count : 1) + 1024;
    fb.reserve(kept * 48);
    foff.reserve(kept + 1);
    fid.reserve(kept);
    src_seed.reserve(p.n_filters);
    std::vector<std::string> lv;
    uint64_t next_id = 0;
    auto keep = [&](uint64_t id) { return p.shard_count <= 1 || shard_mix(id) % p.shard_count == p.shard_index; };
    // The draws from r decide a filter's shape; its words come from its own stream tr.
    // Only the level count (tr's first draw) is needed to replay r, so a filter whose
    // ids all fall in other shards never builds its strings (same output, shards ~G x faster).
    std::vector<uint32_t> plus_at;
    for (uint64_t i = 0; i < p.n_filters; i++) {
        uint64_t sseed = r.next();
        src_seed.push_back(sseed);
        const uint32_t nl = p.min_levels + Rng(sseed).below(p.max_levels - p.min_levels + 1);  // gen_topic's first draw
        bool sys = p.p_sys_filter > 0 && r.uni() < p.p_sys_filter;
        uint32_t sys_node = sys ? r.below(4) : 0;
        std::string f;
        bool hash = r.uni() < p.p_hash;
        bool plus = r.uni() < p.p_plus;
        if (hash && p.plus_hash_excl) plus = false;
        size_t n = nl + (sys ? 3 : 0);
        if (hash) {
            uint32_t d = p.min_hash_depth;
            if (wsum > 0) {
                double u = r.uni() * wsum;
                d = 0;
                while (d < 15 && u >= p.hash_w[d]) u -= p.hash_w[d++];
            } else {
                while (d < n && r.uni() > p.hash_geo) d++;
            }
            if (d > n) d = (uint32_t)n;
            n = d;
        }
        plus_at.clear();
        if (plus) {
            for (size_t k = 0; k < n; k++)
                if (r.uni() < p.p_plus_level) plus_at.push_back((uint32_t)k);
            if (plus_at.empty() && n) plus_at.push_back(r.below((uint32_t)n));
        }
        uint32_t copies = 1;
        if ((hash || plus) && p.p_multi > 0 && r.uni() < p.p_multi) copies += 1 + r.below(p.multi_max ? p.multi_max : 1);
        bool any_kept = false;
        for (uint32_t c = 0; c < copies && !any_kept; c++) any_kept = keep(next_id + c);
        if (!any_kept) {
            next_id += copies;
            continue;
        }
        Rng tr(sseed);
        gen_topic(lv, tr, p, z);
        if (sys) lv.insert(lv.begin(), {"$SYS", "brokers", "emqx@n" + std::to_string(sys_node)});
        for (uint32_t k : plus_at) lv[k] = "+";
        f = joinv(lv, n);
        if (hash) f += n ? "/#" : "#";
        for (uint32_t c = 0; c < copies; c++, next_id++) {
            if (!keep(next_id)) continue;
            fb.insert(fb.end(), f.begin(), f.end());
            foff.push_back(fb.size());
            fid.push_back(next_id);
        }
    }
    // hot '#' filters: a short prefix subscribed by many clients (ids)
    std::vector<uint64_t> hot_seed(p.n_hot);
    std::vector<uint32_t> hot_depth(p.n_hot);
    for (uint32_t h = 0; h < p.n_hot; h++) {
        hot_seed[h] = r.next();
        Rng tr(hot_seed[h]);
        gen_topic(lv, tr, p, z);
        uint32_t span = p.hot_depth_max >= p.hot_depth_min ? p.hot_depth_max - p.hot_depth_min + 1 : 1;
        uint32_t d = p.hot_depth_min + r.below(span);
        if (d > lv.size()) d = (uint32_t)lv.size();
        hot_depth[h] = d;
        std::string f = joinv(lv, d) + (d ? "/#" : "#");
        double lo = std::log((double)std::max(1u, p.hot_ids_min)), hi = std::log((double)std::max(p.hot_ids_min, p.hot_ids_max));
        uint32_t copies = (uint32_t)std::exp(lo + (hi - lo) * r.uni());
        for (uint32_t c = 0; c < copies; c++, next_id++) {
            if (!keep(next_id)) continue;
            fb.insert(fb.end(), f.begin(), f.end());
            foff.push_back(fb.size());
            fid.push_back(next_id);
        }
    }

    std::vector<uint8_t> tb;
    std::vector<uint32_t> toff{0};
    tb.reserve(p.n_topics * 48);
    toff.reserve(p.n_topics + 1);
    for (uint64_t i = 0; i < p.n_topics; i++) {
        if (p.n_hot && r.uni() < p.p_topic_hot) {
            // under a hot prefix: keep its first hot_depth levels, fresh levels below
            uint32_t h = r.below(p.n_hot);
            Rng tr(hot_seed[h]);
            gen_topic(lv, tr, p, z);
            Rng fr(r.next());
            std::vector<std::string> tail;
            gen_topic(tail, fr, p, z);
            for (size_t k = hot_depth[h]; k < lv.size() && k < tail.size(); k++) lv[k] = tail[k];
        } else if (p.p_sys > 0 && r.uni() < p.p_sys) {
            Rng tr(r.next());
            gen_topic(lv, tr, p, z);
            lv.insert(lv.begin(), {"$SYS", "brokers", "emqx@n" + std::to_string(r.below(4))});
        } else if (p.n_filters && r.uni() < p.p_topic_hit) {
            Rng tr(src_seed[r.below((uint32_t)std::min<uint64_t>(p.n_filters, 0xFFFFFFFFu))]);
            gen_topic(lv, tr, p, z);
        } else {
            Rng tr(r.next());
            gen_topic(lv, tr, p, z);
        }
        std::string t = joinv(lv, lv.size());
        if (tb.size() + t.size() > 0xFFFFFFF0ull) return -2;
        tb.insert(tb.end(), t.begin(), t.end());
        toff.push_back((uint32_t)tb.size());
    }

    synth_out *o = new synth_out();
    o->n_keys = fid.size();
    o->f_bytes_len = fb.size();
    o->t_bytes_len = tb.size();
    o->f_bytes = new uint8_t[fb.size() + 16];
    memcpy(o->f_bytes, fb.data(), fb.size());
    memset(o->f_bytes + fb.size(), 0, 16);
    o->f_off = new uint64_t[foff.size()];
    memcpy(o->f_off, foff.data(), foff.size() * 8);
    o->f_id = new uint64_t[fid.size() + 1];
    memcpy(o->f_id, fid.data(), fid.size() * 8);
    o->n_topics = p.n_topics;
    o->t_bytes = new uint8_t[tb.size() + 16];
    memcpy(o->t_bytes, tb.data(), tb.size());
    memset(o->t_bytes + tb.size(), 0, 16);
    o->t_off = new uint32_t[toff.size()];
    memcpy(o->t_off, toff.data(), toff.size() * 4);
    *out = o;
    return 0;
}

void synth_free(synth_out *o) {
    if (!o) return;
    delete[] o->f_bytes;
    delete[] o->f_off;
    delete[] o->f_id;
    delete[] o->t_bytes;
    delete[] o->t_off;
    delete o;
}

}  // extern "C"

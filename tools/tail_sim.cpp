// tail_sim.cpp — CPU estimate of what "single-key tail" path compression would save the walk
// (DESIGN.md §10 lead; development tool, not the product).  Builds the trie of a dumped
// workload (filters split on '/', '+' as its own edge label, a final '#' hangs its key on the
// parent node, as engine.cpp does), counts the keys in every node's subtree, and replays the
// level-synchronous walk of every topic (literal child and '+' child of each frontier node,
// as k_match_fast visits them).  A tail head is a node whose subtree holds exactly one key
// while its parent's holds more; visits to nodes strictly below a head are what a tail record
// at the head (the key's remaining words, compared in registers) would replace.
//
//   g++ -O2 -std=c++17 tools/tail_sim.cpp -o /tmp/tail_sim && /tmp/tail_sim DIR
//   DIR holds fb.bin (filter bytes), fo.bin (u64 offsets), tb.bin, to.bin (u32 offsets).
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <string_view>
#include <unordered_map>
#include <vector>

static std::vector<uint8_t> slurp(const std::string &p) {
    FILE *f = fopen(p.c_str(), "rb");
    if (!f) {
        perror(p.c_str());
        exit(1);
    }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    std::vector<uint8_t> v(n);
    if (fread(v.data(), 1, n, f) != (size_t)n) exit(1);
    fclose(f);
    return v;
}

static constexpr uint32_t PLUS = 0xFFFFFFFEu, NONE = 0xFFFFFFFFu;

struct Trie {
    std::unordered_map<std::string, uint32_t> words;
    std::unordered_map<uint64_t, uint32_t> edge;  // parent << 32 | word -> child
    std::vector<uint32_t> parent, keys;          // per node
    Trie() {
        parent.push_back(NONE);
        keys.push_back(0);
    }
    uint32_t wid(std::string_view w, bool add) {
        auto it = words.find(std::string(w));
        if (it != words.end()) return it->second;
        if (!add) return NONE;
        const uint32_t id = (uint32_t)words.size();
        words.emplace(std::string(w), id);
        return id;
    }
    uint32_t child(uint32_t p, uint32_t w) const {
        auto it = edge.find((uint64_t)p << 32 | w);
        return it == edge.end() ? NONE : it->second;
    }
    uint32_t add_child(uint32_t p, uint32_t w) {
        const uint64_t k = (uint64_t)p << 32 | w;
        auto it = edge.find(k);
        if (it != edge.end()) return it->second;
        const uint32_t c = (uint32_t)parent.size();
        parent.push_back(p);
        keys.push_back(0);
        edge.emplace(k, c);
        return c;
    }
};

static void split(std::string_view s, std::vector<std::string_view> &out) {
    out.clear();
    size_t st = 0;
    for (size_t i = 0; i <= s.size(); i++)
        if (i == s.size() || s[i] == '/') {
            out.push_back(s.substr(st, i - st));
            st = i + 1;
        }
}

int main(int argc, char **argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp/tailsim";
    auto fb = slurp(dir + "/fb.bin"), fo8 = slurp(dir + "/fo.bin"), tb = slurp(dir + "/tb.bin"), to8 = slurp(dir + "/to.bin");
    const uint64_t *fo = (const uint64_t *)fo8.data();
    const uint32_t *to = (const uint32_t *)to8.data();
    const size_t nf = fo8.size() / 8 - 1, nt = to8.size() / 4 - 1;
    Trie T;
    T.edge.reserve(80'000'000);
    std::vector<std::string_view> lv;
    for (size_t i = 0; i < nf; i++) {
        split(std::string_view((const char *)fb.data() + fo[i], fo[i + 1] - fo[i]), lv);
        size_t n = lv.size();
        bool hash = n && lv[n - 1] == "#";
        if (hash) n--;
        bool bad = false;
        for (size_t k = 0; k < n; k++) bad |= lv[k] == "#";
        if (bad) continue;  // '#' before the last level never matches
        uint32_t node = 0;
        for (size_t k = 0; k < n; k++) node = T.add_child(node, lv[k] == "+" ? PLUS : T.wid(lv[k], true));
        T.keys[node]++;  // an exact key ends here, or "node/#" hangs here
    }
    const size_t nn = T.parent.size();
    std::vector<uint64_t> sub(T.keys.begin(), T.keys.end());
    for (size_t v = nn - 1; v > 0; v--) sub[T.parent[v]] += sub[v];  // children come after parents
    // in_tail[v]: v is strictly below a tail head
    std::vector<uint8_t> head(nn, 0), in_tail(nn, 0);
    for (size_t v = 1; v < nn; v++) {
        const uint32_t p = T.parent[v];
        in_tail[v] = (p != 0) && (head[p] || in_tail[p]);
        head[v] = !in_tail[v] && sub[v] == 1;
    }
    uint64_t visits = 0, tail_visits = 0, heads_reached = 0, deep_visits = 0, tail_entries = 0;
    std::vector<uint32_t> fr, nx, wids;
    for (size_t t = 0; t < nt; t++) {
        split(std::string_view((const char *)tb.data() + to[t], to[t + 1] - to[t]), lv);
        wids.clear();
        for (auto w : lv) wids.push_back(T.wid(w, false));
        fr.assign(1, 0);
        for (size_t d = 0; d < wids.size() && !fr.empty(); d++) {
            nx.clear();
            for (uint32_t v : fr) {
                for (uint32_t w : {wids[d], PLUS}) {
                    if (w == NONE) continue;
                    const uint32_t c = T.child(v, w);
                    if (c == NONE) continue;
                    visits++;
                    deep_visits += d >= 4;
                    if (in_tail[c]) {
                        tail_visits++;
                        tail_entries += head[T.parent[c]];  // the first tail node below its head
                    }
                    else if (head[c]) heads_reached++;
                    nx.push_back(c);
                }
            }
            fr.swap(nx);
        }
    }
    printf("{\"filters\": %zu, \"topics\": %zu, \"nodes\": %zu, \"tail_heads\": %llu, \"nodes_in_tails\": %llu, "
           "\"visits\": %llu, \"visits_in_tails\": %llu, \"tail_entries\": %llu, \"tail_heads_reached\": %llu, "
           "\"visits_depth_ge4\": %llu}\n",
           nf, nt, nn, (unsigned long long)std::count(head.begin(), head.end(), 1),
           (unsigned long long)std::count(in_tail.begin(), in_tail.end(), 1), (unsigned long long)visits,
           (unsigned long long)tail_visits, (unsigned long long)tail_entries, (unsigned long long)heads_reached,
           (unsigned long long)deep_visits);
    return 0;
}

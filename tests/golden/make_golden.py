"""Writes the golden fixtures in tests/golden/.

Two kinds of vectors:

1. Known-answer cases transcribed BY HAND from the reference's own test suites (the
   expected values below are the reference's assertions, copied as data; file:line
   cites the assertion).  These pin the oracle and the engine independently of any
   code written here.
2. `config_a_sample.json`: a small seeded sample of BASELINE config A whose expected
   match sets come from the brute-force emqx_topic:match/2 restatement
   (oracle/trie_search.cpp, algo=brute) — cross-checked against the pure-Python
   restatement (oracle/emqx_topic.py) before writing.  Regenerate with
   `python tests/golden/make_golden.py`.
"""
from __future__ import annotations

import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))

T = "a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q/r/s/t/u/v/w/x/y/z"

# ---------------------------------------------------------------------------
# emqx_topic:match/2 — apps/emqx/test/emqx_topic_SUITE.erl
TOPIC_MATCH = [
    # t_match1 :53-66
    ["a/b/c", "a/b/+", True], ["a/b/c", "a/#", True], ["abcd/ef/g", "#", True],
    ["abc/de/f", "abc/de/f", True], ["abc", "+", True], ["a/b/c", "a/b/c", True],
    ["a/b/c", "a/c/d", False], ["$share/x/y", "+", False], ["$share/x/y", "+/x/y", False],
    ["$share/x/y", "#", False], ["$share/x/y", "+/+/#", False],
    ["house/1/sensor/0", "house/+", False], ["house", "house/+", False],
    # t_match2 :68-85
    ["sport/tennis/player1", "sport/tennis/player1/#", True],
    ["sport/tennis/player1/ranking", "sport/tennis/player1/#", True],
    ["sport/tennis/player1/score/wimbledon", "sport/tennis/player1/#", True],
    ["sport", "sport/#", True], ["sport", "#", True], ["/sport/football/score/1", "#", True],
    ["Topic/C", "+/+", True], ["TopicA/B", "+/+", True], ["TopicA/C", "+/+", True],
    ["abc", "+", True], ["a/b/c", "a/b/c", True], ["a/b/c", "a/c/d", False],
    ["$share/x/y", "+", False], ["$share/x/y", "+/x/y", False], ["$share/x/y", "#", False],
    ["$share/x/y", "+/+/#", False], ["house/1/sensor/0", "house/+", False],
    # t_match3 :87-93
    ["device/60019423a83c/fw", "device/60019423a83c/#", True],
    ["device/60019423a83c/$fw", "device/60019423a83c/#", True],
    ["device/60019423a83c/$fw/fw", "device/60019423a83c/$fw/#", True],
    ["device/60019423a83c/fw/checksum", "device/60019423a83c/#", True],
    ["device/60019423a83c/$fw/checksum", "device/60019423a83c/#", True],
    ["device/60019423a83c/dust/type", "device/60019423a83c/#", True],
    # t_sigle_level_match :95-104
    ["sport/tennis/player1", "sport/tennis/+", True],
    ["sport/tennis/player1/ranking", "sport/tennis/+", False],
    ["sport", "sport/+", False], ["sport/", "sport/+", True],
    ["/finance", "+/+", True], ["/finance", "/+", True], ["/finance", "+", False],
    ["/devices/$dev1", "/devices/+", True], ["/devices/$dev1/online", "/devices/+/online", True],
    # t_sys_match :106-110
    ["$SYS/broker/clients/testclient", "$SYS/#", True], ["$SYS/broker", "$SYS/+", True],
    ["$SYS/broker", "+/+", False], ["$SYS/broker", "#", False],
    # 't_#_match' :112-117
    ["a/b/c", "#", True], ["a/b/c", "+/#", True], ["$SYS/brokers", "#", False],
    ["a/b/$c", "a/b/#", True], ["a/b/$c", "a/#", True],
    # t_match_perf :125-130
    ["a/b/ccc", "a/#", True],
    ["/abkc/19383/192939/akakdkkdkak/xxxyyuya/akakak", "/abkc/19383/+/akakdkkdkak/#", True],
]
# t_match_tokens :119-123 — raw tokens (empty level stays <<>>) vs words (empty -> '')
TOPIC_MATCH_TOKENS = [["a/b/c", "a/+/c", True], ["a//c", "a/+/c", True], ["a//c/", "a/+/c", False],
                      ["a//c/", "a/+/c/#", True]]

TOPIC_MISC = {
    # t_wildcard :47-51
    "wildcard": [["a/b/#", True], ["a/+/#", True], ["", False], ["a/b/c", False]],
    # t_validate :189-232, t_sigle_level_validate :234-238  [kind, topic, expected | error]
    "validate": [
        ["filter", "a/+/#", True], ["filter", "a/b/c/d", True], ["name", "abc/de/f", True],
        ["filter", "abc/+/f", True], ["filter", "abc/#", True], ["filter", "x", True],
        ["name", "x//y", True], ["filter", "sport/tennis/#", True],
        ["name", "", "empty_topic"], ["filter", "", "empty_topic"], ["name", "abc/#", "topic_name_error"],
        ["filter", "abc/#xzy/+", "topic_invalid_char"], ["filter", "abc/xzy/+9827", "topic_invalid_char"],
        ["filter", "sport/tennis#", "topic_invalid_char"], ["filter", "abc/#/1", "topic_invalid_#"],
        ["filter", "sport/tennis/#/ranking", "topic_invalid_#"],
        ["filter", "$share/", "share_empty_filter"], ["filter", "$share//", "share_empty_filter"],
        ["filter", "$share//t", "share_empty_group"], ["filter", "$share//test", "share_empty_group"],
        ["filter", "$share/g/", "share_empty_filter"], ["filter", "$share/g2/", "share_empty_filter"],
        ["filter", "$share/p+q/1", "share_name_invalid_char"], ["filter", "$share/m+/1", "share_name_invalid_char"],
        ["filter", "$share/+n/1", "share_name_invalid_char"], ["filter", "$share/x#y/1", "share_name_invalid_char"],
        ["filter", "$share/x#/1", "share_name_invalid_char"], ["filter", "$share/#y/1", "share_name_invalid_char"],
        ["filter", "$share/g1/$share/t", "share_recursively"], ["filter", "$share/g1/topic/$share", True],
        ["filter", "+", True], ["filter", "+/tennis/#", True], ["filter", "sport/+/player1", True],
        ["filter", "sport+", "topic_invalid_char"],
    ],
    # t_levels :247-249 ; t_tokens :251-255
    "levels": [["a/+/#", 3], ["a/b/c/d", 4]],
    "tokens": [["a/b/+/#", ["a", "b", "+", "#"]]],
    # t_words :257-263   (atoms written as {"atom": name})
    "words": [["/a/+/#", [{"atom": ""}, "a", {"atom": "+"}, {"atom": "#"}]],
              ["/abkc/19383/+/akakdkkdkak/#", [{"atom": ""}, "abkc", "19383", {"atom": "+"}, "akakdkkdkak",
                                               {"atom": "#"}]]],
    # t_join :265-276
    "join": [[[], ""], [["x"], "x"], [[{"atom": "#"}], "#"], [[{"atom": "+"}, {"atom": ""}, {"atom": "#"}], "+//#"],
             [["x", "y", "z", {"atom": "+"}], "x/y/z/+"], ["@words:/ab/cd/ef/", "/ab/cd/ef/"],
             ["@words:ab/+/#", "ab/+/#"],
             [[{"atom": "+"}, "a", {"atom": "#"}, "b", {"atom": ""}, {"atom": "+"}], {"error": "topic_invalid_#"}],
             [[{"atom": "+"}, "c", "#", "d", {"atom": ""}, {"atom": "+"}], {"error": "topic_invalid_#"}]],
    # emqx_topic_SUITE intersection KATs, every assertion; t_intersect_commutes :148-181 is
    # the argument swap, checked for every row by the tests
    "intersection": [
        # t_intersect :132-139
        ["t/global/#", "t/+/1/+", "t/global/1/+"], ["t/global/#", "#", "t/global/#"],
        ["t/global/#", "t/global/#", "t/global/#"], ["1/+/3/+/5/#", "+/2/+/4/+", "1/2/3/4/5"],
        ["t/local/1/#", "t/local/+", "t/local/1"], ["t/global/#", "t/local/+", False],
        ["t/local/1/+", "t/local/+", False],
        # t_intersect_topic_wildcard :141-147
        ["t/test/#", "t/test/1", "t/test/1"], ["t/test/1/1", "t/test/#", "t/test/1/1"],
        ["t/test/1/1", "t/test/+", False], ["t/test/1/1", "t/test/1/1", "t/test/1/1"],
        ["t/test/1", "t/test/2", False], ["t/test/1", "t/test/1/2", False],
        # t_sys_intersect :183-187
        ["$SYS/broker/#", "$SYS/+/+", "$SYS/broker/+"], ["$SYS/broker", "$SYS/+", "$SYS/broker"],
        ["$SYS/broker", "+/+", False], ["$SYS/broker", "#", False]],
    # emqx_trie_search_tests:filter_test_ :23-33 — filter/1: the key words of a wildcard
    # filter (empty level stays <<>>), false for a filter without wildcards
    "filter": [["sensor/+/metric//#", ["sensor", {"atom": "+"}, "metric", "", {"atom": "#"}]],
               ["sensor/1/metric//42", False]],
    # t_prepend :240-245
    "prepend": [[None, "ab", "ab"], ["", "a/b", "a/b"], ["x/", "a/b", "x/a/b"], ["x/y", "a/b", "x/y/a/b"],
                [{"atom": "+"}, "a/b", "+/a/b"]],
    # t_parse :302-331   [input, expected {"share": [g, t]} | topic | {"error": ...}]
    "parse": [["$share/t", {"error": "invalid_topic_filter"}], ["$share/+/t", {"error": "invalid_topic_filter"}],
              ["a/b/+/#", "a/b/+/#"], ["$queue/topic", {"share": ["$queue", "topic"]}],
              ["$share/group/topic", {"share": ["group", "topic"]}], ["$local/topic", "$local/topic"],
              ["$local/$queue/topic", "$local/$queue/topic"],
              ["$local/$share/group/a/b/c", "$local/$share/group/a/b/c"], ["$fastlane/topic", "$fastlane/topic"]],
}

# ---------------------------------------------------------------------------
# emqx_topic_index — apps/emqx/test/emqx_topic_index_SUITE.erl (+ emqx_trie_SUITE, v1)
# insert: [filter, id] or [filter_words_list, id] ; query kinds:
#   "matches_topics": sorted get_topic of matches(T, [])      (list compare)
#   "matches_ids":    ids of matches(T, opts) in returned order (unique: ordered by id)
#   "match_id" / "match_topic": match/2 (return_first) ; false -> null
#   "count": length(matches(T, []))
#   "badarg": the topic raises badarg
INDEX_CASES = [
    {"name": "t_insert :51-58", "insert": [["sensor/1/metric/2", "t_insert_1"], ["sensor/+/#", "t_insert_2"],
                                           ["sensor/#", "t_insert_3"]],
     "queries": [["match_topic", "sensor", "sensor/#"], ["match_id", "sensor", "t_insert_3"]]},
    {"name": "t_insert_filter :60-69", "insert": [["sensor/+/metric//#", 1],
                                                  [["sensor", {"atom": "+"}, "metric", "", {"atom": "#"}], 2]],
     "queries": [["matches_topics", "sensor/1/metric//2", ["sensor/+/metric//#", "sensor/+/metric//#"]]]},
    {"name": "t_match :71-80", "insert": [["sensor/1/metric/2", "t_match_1"], ["sensor/+/#", "t_match_2"],
                                          ["sensor/#", "t_match_3"]],
     "queries": [["matches_topics", "sensor/1", ["sensor/#", "sensor/+/#"]]]},
    {"name": "t_match2 :82-99", "insert": [["#", "t_match2_1"], ["+/#", "t_match2_2"], ["+/+/#", "t_match2_3"]],
     "queries": [["matches_topics", "a/b/c", ["#", "+/#", "+/+/#"]], ["match_id", "$SYS/broker/zenmq", None],
                 ["matches_topics", "$SYS/broker/zenmq", []]]},
    {"name": "t_match3 :101-123", "insert": [["d/#", "t_match3_1"], ["a/b/+", "t_match3_2"], ["a/#", "t_match3_3"],
                                             ["#", "t_match3_4"], ["$SYS/#", "t_match3_sys"]],
     "queries": [["count", "a/b/c", 3], ["match_id", "$SYS/a/b/c", "t_match3_sys"]]},
    {"name": "t_match4 :125-140", "insert": [["/#", "t_match4_1"], ["/+", "t_match4_2"], ["/+/a/b/c", "t_match4_3"]],
     "queries": [["matches_topics", "/", ["/#", "/+"]], ["matches_topics", "/0/a/b/c", ["/#", "/+/a/b/c"]]]},
    {"name": "t_match5 :142-162", "insert": [["#", "t_match5_1"], [T + "/#", "t_match5_2"], [T + "/+", "t_match5_3"]],
     "queries": [["matches_topics", T, ["#", T + "/#"]], ["matches_topics", T + "/1", ["#", T + "/#", T + "/+"]]]},
    {"name": "t_match6 :164-170", "insert": [["+/" * 26 + "#", "t_match6"]],
     "queries": [["match_id", T, "t_match6"]]},
    {"name": "t_match7 :172-178", "insert": [["a/+/c/+/e/+/g/+/i/+/k/+/m/+/o/+/q/+/s/+/u/+/w/+/y/+/#", "t_match7"]],
     "queries": [["match_topic", T, "a/+/c/+/e/+/g/+/i/+/k/+/m/+/o/+/q/+/s/+/u/+/w/+/y/+/#"]]},
    {"name": "t_match8 :180-204", "insert": [[f, i] for f in ["+", "dev/global/sensor", "dev/+/sensor/#"]
                                             for i in [1, 2, 3]],
     "queries": [["matches_topics", "dev/global/sensor",
                  ["dev/+/sensor/#"] * 3 + ["dev/global/sensor"] * 3]]},
    {"name": "t_match_fast_forward :206-213", "insert": [["a/b/1/2/3/4/5/6/7/8/9/#", "id1"], ["z/y/x/+/+", "id2"],
                                                         ["a/b/c/+", "id3"]],
     "queries": [["match_id", "a/b/1/2/3/4/5/6/7/8/9/0", "id1"], ["matches_ids", "a/b/1/2/3/4/5/6/7/8/9/0", [], ["id1"]]]},
    {"name": "t_match_unique :215-228", "insert": [["a/b/c", "t_match_id1"], ["a/b/+", "t_match_id1"],
                                                   ["a/b/c/+", "t_match_id2"]],
     "queries": [["matches_ids", "a/b/c", [], ["t_match_id1", "t_match_id1"]],
                 ["matches_ids", "a/b/c", ["unique"], ["t_match_id1"]]]},
    # t_match_wildcard_edge_cases :230-265 (ids are 1-based list positions)
    {"name": "t_match_wildcard_edge_cases :245", "insert": [[t, i + 1] for i, t in enumerate(
        ["a/b", "a/b/#", "a/b/#", "a/b/c", "a/b/+", "a/b/d", "a/+/+", "a/+/#"])],
     "queries": [["match_id", "a/b/c", 8], ["matches_ids", "a/b/c", ["unique"], [2, 3, 4, 5, 7, 8]]]},
    {"name": "t_match_wildcard_edge_cases :246", "insert": [[t, i + 1] for i, t in enumerate(
        ["a/b", "a/b/#", "a/b/#", "a/b/c", "a/b/+", "a/b/d", "a/+/+", "a/+/#"])],
     "queries": [["match_id", "a/b", 8], ["matches_ids", "a/b", ["unique"], [1, 2, 3, 8]]]},
    {"name": "t_match_wildcard_edge_cases :247", "insert": [["+/b/c", 1], ["/", 2]],
     "queries": [["match_id", "a/b/c", 1], ["matches_ids", "a/b/c", ["unique"], [1]]]},
    {"name": "t_match_wildcard_edge_cases :248", "insert": [["#", 1], ["/", 2]],
     "queries": [["match_id", "a", 1], ["matches_ids", "a", ["unique"], [1]]]},
    {"name": "t_match_wildcard_edge_cases :249", "insert": [["/", 1], ["+", 2]],
     "queries": [["match_id", "a", 2], ["matches_ids", "a", ["unique"], [2]]]},
    {"name": "t_prop_edgecase :267-278", "insert": [["", 1], ["+/01", 2], ["", 3], ["+/+/01", 4]],
     "queries": [["matches_ids", "01/01", ["unique"], [2]]]},
    # emqx_trie_search_tests:topic_validation_test_ :29-46 (empty index)
    {"name": "trie_search_tests topic_validation", "insert": [],
     "queries": [["badarg", "+"], ["badarg", "#"], ["badarg", "a/+/b"], ["badarg", "a/b/#"],
                 ["match_id", "a/b/b+", None], ["match_id", "a/b/c#", None]]},
    # emqx_trie_SUITE (routing schema v1) :63-187 — same semantics on the index
    {"name": "emqx_trie_SUITE t_match4 :109-113", "insert": [["/#", 1], ["/+", 2], ["/+/a/b/c", 3]],
     "queries": [["matches_topics", "/0/a/b/c", ["/#", "/+/a/b/c"]]]},
    {"name": "emqx_trie_SUITE t_match3 :98-107", "insert": [[t, i] for i, t in enumerate(
        ["d/#", "a/b/+", "a/#", "#", "$SYS/#"])],
     "queries": [["count", "a/b/c", 3], ["matches_topics", "$SYS/a/b/c", ["$SYS/#"]]]},
    {"name": "emqx_trie_SUITE t_match6 :127-131", "insert": [["+/" * 26 + "#", 1]],
     "queries": [["matches_topics", T, ["+/" * 26 + "#"]]]},
    {"name": "emqx_trie_SUITE t_delete :147-160", "insert": [["sensor/1/#", 1], ["sensor/1/metric/2", 1],
                                                            ["sensor/1/metric/3", 1]],
     "delete": [["sensor/1/metric/2", 1], ["sensor/1/metric", 1], ["sensor/1/metric", 1]],
     "queries": [["matches_topics", "sensor/1/x", ["sensor/1/#"]]]},
    {"name": "emqx_trie_SUITE t_delete2 :162-175", "insert": [["sensor", 1], ["sensor/1/metric/2", 1],
                                                             ["sensor/+/metric/3", 1]],
     "delete": [["sensor", 1], ["sensor/1/metric/2", 1], ["sensor/+/metric/3", 1], ["sensor/+/metric/3", 1]],
     "queries": [["matches_topics", "sensor", []], ["matches_topics", "sensor/1", []]]},
    {"name": "emqx_trie_SUITE t_delete3 :177-191", "insert": [["sensor/+", 1], ["sensor/+/metric/2", 1],
                                                             ["sensor/+/metric/3", 1]],
     "delete": [["sensor/+/metric/2", 1], ["sensor/+/metric/3", 1], ["sensor", 1], ["sensor/+", 1],
                ["sensor/+/unknown", 1]],
     "queries": [["matches_topics", "sensor", []]]},
]

# ---------------------------------------------------------------------------
# emqx_router (schema v2) — apps/emqx/test/emqx_router_SUITE.erl ; shared subs —
# apps/emqx/test/emqx_shared_sub_SUITE.erl:1017-1052.  Steps: ["add"|"del", topic, dest]
# or ["match", topic, sorted [[filter, dest], ...]]; dest "node" = node().
ROUTER_CASES = [
    {"name": "t_add_delete_incremental :88-135", "steps": [
        ["add", "a/b/c", "node"], ["add", "a/+/c", "node"], ["add", "a/+/+", "node"], ["add", "a/b/#", "node"],
        ["add", "#", "node"],
        ["match", "a/b/c", [["#", "node"], ["a/+/+", "node"], ["a/+/c", "node"], ["a/b/#", "node"],
                            ["a/b/c", "node"]]],
        ["del", "a/+/c", "node"],
        ["match", "a/b/c", [["#", "node"], ["a/+/+", "node"], ["a/b/#", "node"], ["a/b/c", "node"]]],
        ["del", "a/+/+", "node"],
        ["match", "a/b/c", [["#", "node"], ["a/b/#", "node"], ["a/b/c", "node"]]],
        ["del", "a/b/#", "node"],
        ["match", "a/b/c", [["#", "node"], ["a/b/c", "node"]]],
        ["del", "a/b/c", "node"],
        ["match", "a/b/c", [["#", "node"]]]]},
    {"name": "t_match_routes :147-165", "steps": [
        ["add", "a/b/c", "node"], ["add", "a/+/c", "node"], ["add", "a/b/#", "node"], ["add", "#", "node"],
        ["match", "a/b/c", [["#", "node"], ["a/+/c", "node"], ["a/b/#", "node"], ["a/b/c", "node"]]],
        ["del", "a/b/c", "node"], ["del", "a/+/c", "node"], ["del", "a/b/#", "node"], ["del", "#", "node"],
        ["match", "a/b/c", []]]},
    {"name": "t_add_delete :80-86 (topics)", "steps": [
        ["add", "a/b/c", "node"], ["add", "a/b/c", "node"], ["add", "a/+/b", "node"],
        ["topics", ["a/+/b", "a/b/c"]], ["del", "a/b/c", "node"], ["del", "a/+/b", "node"], ["topics", []]]},
    # t_queue_subscription :1120-1137: $queue/t/1 and $share/aa/t/1 are two routes on t/1
    # (groups '$queue' and 'aa', emqx_topic:parse/1 :342-354; emqx_shared_sub.erl:450)
    {"name": "emqx_shared_sub_SUITE t_queue_subscription :1120-1137", "steps": [
        ["sub", "$queue/t/1", "node"], ["sub", "$share/aa/t/1", "node"],
        ["count", "t/1", 2],
        ["match", "t/1", [["t/1", ["$queue", "node"]], ["t/1", ["aa", "node"]]]]]},
    {"name": "emqx_shared_sub_SUITE two groups :1017-1052", "steps": [
        ["add", "t/1", ["g1", "node"]], ["add", "t/1", ["g2", "node"]],
        ["match", "t/1", [["t/1", ["g1", "node"]], ["t/1", ["g2", "node"]]]]]},
]


def dump(name, obj):
    with open(os.path.join(HERE, name), "w") as f:
        json.dump(obj, f, indent=1, sort_keys=True)
        f.write("\n")


def config_a_sample():
    sys.path.insert(0, ROOT)
    import numpy as np

    import oracle
    from emqx_amd import workloads
    from oracle import emqx_topic as et

    w = workloads.generate("A", scale=0.2, n_topics=400)   # 2,000 keys, 400 topics
    ix = oracle.OrderedIndex(w.f_bytes, w.f_off, w.f_id)
    off, ids, st = ix.match(w.t_bytes, w.t_off, algo=oracle.ALGO_BRUTE)
    filters = w.filters()
    topics = w.topics()
    # cross-check the C brute force with the Python restatement
    for i, t in enumerate(topics):
        exp = sorted(int(w.f_id[k]) for k, f in enumerate(filters) if et.match(t, f))
        got = ids[off[i]:off[i + 1]].tolist()
        assert exp == got, (t, exp, got)
    return {
        "about": "BASELINE config A, scale 0.2 (seed 0xE11A0001): expected = brute-force emqx_topic:match/2",
        "filters": [f.decode() for f in filters], "ids": [int(x) for x in w.f_id],
        "topics": [t.decode() for t in topics],
        "expected": [ids[off[i]:off[i + 1]].tolist() for i in range(len(topics))],
    }


if __name__ == "__main__":
    dump("kat_topic.json", {"match": TOPIC_MATCH, "match_tokens": TOPIC_MATCH_TOKENS, **TOPIC_MISC})
    dump("kat_index.json", INDEX_CASES)
    dump("kat_router.json", ROUTER_CASES)
    dump("config_a_sample.json", config_a_sample())
    print("golden fixtures written")

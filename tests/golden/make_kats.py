"""Writes tests/golden/kats.json: the reference's own known-answer tests for the
route-lookup path, transcribed as DATA (inputs + the expected outputs the reference
tests assert).  Each case cites the reference file:line it comes from
(paths relative to /root/reference).

Run:  python tests/golden/make_kats.py   (deterministic; the JSON is committed)
"""

import json
import os

T26 = "a/b/c/d/e/f/g/h/i/j/k/l/m/n/o/p/q/r/s/t/u/v/w/x/y/z"

# ---------------------------------------------------------------------------
# emqx_trie_SUITE (every case runs in both groups compact / not_compact,
# emqx_trie_SUITE.erl:27-41).  ops: ["insert"|"delete", filter]; queries: topic ->
# expected sorted match list.  Cases that assert only a length carry "expect_len".
# ---------------------------------------------------------------------------
TRIE_CASES = [
    {"name": "t_insert", "src": "apps/emqx/test/emqx_trie_SUITE.erl:63-70",
     "ops": [["insert", "sensor/1/metric/2"], ["insert", "sensor/+/#"], ["insert", "sensor/#"]],
     "queries": [["sensor", ["sensor/#"]]]},
    {"name": "t_match", "src": "apps/emqx/test/emqx_trie_SUITE.erl:72-79",
     "ops": [["insert", "sensor/1/metric/2"], ["insert", "sensor/+/#"], ["insert", "sensor/#"]],
     "queries": [["sensor/1", ["sensor/#", "sensor/+/#"]]]},
    {"name": "t_match_invalid", "src": "apps/emqx/test/emqx_trie_SUITE.erl:81-88",
     "ops": [["insert", "sensor/1/metric/2"], ["insert", "sensor/+/#"], ["insert", "sensor/#"]],
     "queries": [["sensor/+", []], ["#", []]]},
    {"name": "t_match2", "src": "apps/emqx/test/emqx_trie_SUITE.erl:91-99",
     "ops": [["insert", "#"], ["insert", "+/#"], ["insert", "+/+/#"]],
     "queries": [["a/b/c", ["#", "+/#", "+/+/#"]], ["$SYS/broker/zenmq", []]]},
    {"name": "t_match3", "src": "apps/emqx/test/emqx_trie_SUITE.erl:101-110",
     "ops": [["insert", t] for t in ["d/#", "a/b/+", "a/#", "#", "$SYS/#"]],
     "queries": [["$SYS/a/b/c", ["$SYS/#"]]],
     "len_queries": [["a/b/c", 3]]},
    {"name": "t_match4", "src": "apps/emqx/test/emqx_trie_SUITE.erl:112-115",
     "ops": [["insert", t] for t in ["/#", "/+", "/+/a/b/c"]],
     "queries": [["/0/a/b/c", ["/#", "/+/a/b/c"]]]},
    {"name": "t_match5", "src": "apps/emqx/test/emqx_trie_SUITE.erl:117-123",
     "ops": [["insert", t] for t in ["#", T26 + "/#", T26 + "/+"]],
     "queries": [[T26, ["#", T26 + "/#"]],
                 [T26 + "/1", ["#", T26 + "/#", T26 + "/+"]]]},
    {"name": "t_match6", "src": "apps/emqx/test/emqx_trie_SUITE.erl:125-129",
     "ops": [["insert", "+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/#"]],
     "queries": [[T26, ["+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/+/#"]]]},
    {"name": "t_match7", "src": "apps/emqx/test/emqx_trie_SUITE.erl:131-135",
     "ops": [["insert", "a/+/c/+/e/+/g/+/i/+/k/+/m/+/o/+/q/+/s/+/u/+/w/+/y/+/#"]],
     "queries": [[T26, ["a/+/c/+/e/+/g/+/i/+/k/+/m/+/o/+/q/+/s/+/u/+/w/+/y/+/#"]]]},
    {"name": "t_empty", "src": "apps/emqx/test/emqx_trie_SUITE.erl:137-142",
     "ops": [["assert_empty", True], ["insert", "topic/x/#"], ["assert_empty", False],
             ["delete", "topic/x/#"], ["assert_empty", True]],
     "queries": []},
    {"name": "t_delete", "src": "apps/emqx/test/emqx_trie_SUITE.erl:144-155",
     "ops": [["insert", "sensor/1/#"], ["insert", "sensor/1/metric/2"], ["insert", "sensor/1/metric/3"],
             ["delete", "sensor/1/metric/2"], ["delete", "sensor/1/metric"], ["delete", "sensor/1/metric"]],
     "queries": [["sensor/1/x", ["sensor/1/#"]]]},
    {"name": "t_delete2", "src": "apps/emqx/test/emqx_trie_SUITE.erl:157-170",
     "ops": [["insert", "sensor"], ["insert", "sensor/1/metric/2"], ["insert", "sensor/+/metric/3"],
             ["delete", "sensor"], ["delete", "sensor/1/metric/2"], ["delete", "sensor/+/metric/3"],
             ["delete", "sensor/+/metric/3"]],
     "queries": [["sensor", []], ["sensor/1", []]]},
    {"name": "t_delete3", "src": "apps/emqx/test/emqx_trie_SUITE.erl:172-186",
     "ops": [["insert", "sensor/+"], ["insert", "sensor/+/metric/2"], ["insert", "sensor/+/metric/3"],
             ["delete", "sensor/+/metric/2"], ["delete", "sensor/+/metric/3"], ["delete", "sensor"],
             ["delete", "sensor/+"], ["delete", "sensor/+/unknown"]],
     "queries": [["sensor", []]],
     "lookup_topic": [["sensor/+", []]]},
]

# eunit in emqx_trie.erl (TEST section).  Keys: [binary, 0|1].
EUNIT = {
    "make_keys": {
        "src": "apps/emqx/src/emqx_trie.erl:345-361",
        "no_compact": [["#", ["#", 1], []], ["a/+", ["a/+", 1], [["a", 0]]], ["+", ["+", 1], []]],
        "compact": [["#", ["#", 1], []], ["a/+", ["a/+", 1], []], ["+", ["+", 1], []],
                    ["a/+/c", ["a/+/c", 1], [["a/+", 0]]]],
    },
    "make_prefixes": {
        "src": "apps/emqx/src/emqx_trie.erl:374-386",
        "no_compact": [["a/b/+", ["a/b", "a"]], ["a/b/+/c/#", ["a/b/+/c", "a/b/+", "a/b", "a"]]],
        "compact": [["a/b/+", []], ["a/b/+/c/#", ["a/b/+"]]],
    },
    "do_compact": {
        "src": "apps/emqx/src/emqx_trie.erl:388-395",
        "cases": [["/+", ["/+"]], ["/#", ["/#"]], ["a/b/+/c", ["a/b/+", "c"]],
                  ["a/+/+/b", ["a/+", "+", "b"]], ["a/+/+/+/+/b", ["a/+", "+", "+", "+", "b"]]],
    },
}

# emqx_topic_SUITE: match/2 pairs [name, filter, expected]
TOPIC_MATCH = [
    # t_match1  emqx_topic_SUITE.erl:48-61
    ["a/b/c", "a/b/+", True], ["a/b/c", "a/#", True], ["abcd/ef/g", "#", True],
    ["abc/de/f", "abc/de/f", True], ["abc", "+", True], ["a/b/c", "a/b/c", True],
    ["a/b/c", "a/c/d", False], ["$share/x/y", "+", False], ["$share/x/y", "+/x/y", False],
    ["$share/x/y", "#", False], ["$share/x/y", "+/+/#", False],
    ["house/1/sensor/0", "house/+", False], ["house", "house/+", False],
    # t_match2  :63-80
    ["sport/tennis/player1", "sport/tennis/player1/#", True],
    ["sport/tennis/player1/ranking", "sport/tennis/player1/#", True],
    ["sport/tennis/player1/score/wimbledon", "sport/tennis/player1/#", True],
    ["sport", "sport/#", True], ["sport", "#", True], ["/sport/football/score/1", "#", True],
    ["Topic/C", "+/+", True], ["TopicA/B", "+/+", True], ["TopicA/C", "+/+", True],
    ["abc", "+", True], ["a/b/c", "a/b/c", True], ["a/b/c", "a/c/d", False],
    ["$share/x/y", "+", False], ["$share/x/y", "+/x/y", False], ["$share/x/y", "#", False],
    ["$share/x/y", "+/+/#", False], ["house/1/sensor/0", "house/+", False],
    # t_match3  :82-88
    ["device/60019423a83c/fw", "device/60019423a83c/#", True],
    ["device/60019423a83c/$fw", "device/60019423a83c/#", True],
    ["device/60019423a83c/$fw/fw", "device/60019423a83c/$fw/#", True],
    ["device/60019423a83c/fw/checksum", "device/60019423a83c/#", True],
    ["device/60019423a83c/$fw/checksum", "device/60019423a83c/#", True],
    ["device/60019423a83c/dust/type", "device/60019423a83c/#", True],
    # t_sigle_level_match  :90-99
    ["sport/tennis/player1", "sport/tennis/+", True],
    ["sport/tennis/player1/ranking", "sport/tennis/+", False],
    ["sport", "sport/+", False], ["sport/", "sport/+", True], ["/finance", "+/+", True],
    ["/finance", "/+", True], ["/finance", "+", False], ["/devices/$dev1", "/devices/+", True],
    ["/devices/$dev1/online", "/devices/+/online", True],
    # t_sys_match  :101-105
    ["$SYS/broker/clients/testclient", "$SYS/#", True], ["$SYS/broker", "$SYS/+", True],
    ["$SYS/broker", "+/+", False], ["$SYS/broker", "#", False],
    # t_#_match  :107-112
    ["a/b/c", "#", True], ["a/b/c", "+/#", True], ["$SYS/brokers", "#", False],
    ["a/b/$c", "a/b/#", True], ["a/b/$c", "a/#", True],
    # t_match_perf  :114-118
    ["a/b/ccc", "a/#", True],
    ["/abkc/19383/192939/akakdkkdkak/xxxyyuya/akakak", "/abkc/19383/+/akakdkkdkak/#", True],
]

TOPIC_MISC = {
    "wildcard": {"src": "apps/emqx/test/emqx_topic_SUITE.erl:42-46",
                 "cases": [["a/b/#", True], ["a/+/#", True], ["", False], ["a/b/c", False]]},
    "words": {"src": "apps/emqx/test/emqx_topic_SUITE.erl:160-163",
              "cases": [["/a/+/#", ["''", "a", "'+'", "'#'"]],
                        ["/abkc/19383/+/akakdkkdkak/#",
                         ["''", "abkc", "19383", "'+'", "akakdkkdkak", "'#'"]]]},
    "tokens": {"src": "apps/emqx/test/emqx_topic_SUITE.erl:156-158",
               "cases": [["a/b/+/#", ["a", "b", "+", "#"]]]},
    "levels": {"src": "apps/emqx/test/emqx_topic_SUITE.erl:152-154",
               "cases": [["a/+/#", 3], ["a/b/c/d", 4]]},
    "join": {"src": "apps/emqx/test/emqx_topic_SUITE.erl:168-175",
             "cases": [[[], ""], [["x"], "x"], [["'#'"], "#"], [["'+'", "''", "'#'"], "+//#"],
                       [["x", "y", "z", "'+'"], "x/y/z/+"],
                       [{"words_of": "/ab/cd/ef/"}, "/ab/cd/ef/"],
                       [{"words_of": "ab/+/#"}, "ab/+/#"]]},
    "validate_ok": {"src": "apps/emqx/test/emqx_topic_SUITE.erl:121-129,139-142",
                    "cases": [["filter", "a/+/#"], ["filter", "a/b/c/d"], ["name", "abc/de/f"],
                              ["filter", "abc/+/f"], ["filter", "abc/#"], ["filter", "x"],
                              ["name", "x//y"], ["filter", "sport/tennis/#"], ["filter", "+"],
                              ["filter", "+/tennis/#"], ["filter", "sport/+/player1"]]},
    "validate_err": {"src": "apps/emqx/test/emqx_topic_SUITE.erl:130-137,143",
                     "cases": [["name", "", "empty_topic"], ["name", "abc/#", "topic_name_error"],
                               ["name", {"long_topic": True}, "topic_too_long"],
                               ["filter", "abc/#/1", "topic_invalid_#"],
                               ["filter", "abc/#xzy/+", "topic_invalid_char"],
                               ["filter", "abc/xzy/+9827", "topic_invalid_char"],
                               ["filter", "sport/tennis#", "topic_invalid_char"],
                               ["filter", "sport/tennis/#/ranking", "topic_invalid_#"],
                               ["filter", "sport+", "topic_invalid_char"]]},
    "prepend": {"src": "apps/emqx/test/emqx_topic_SUITE.erl:145-150",
                "cases": [[None, "ab", "ab"], ["", "a/b", "a/b"], ["x/", "a/b", "x/a/b"],
                          ["x/y", "a/b", "x/y/a/b"], ["'+'", "a/b", "+/a/b"]]},
    "feed_var": {"src": "apps/emqx/test/emqx_topic_SUITE.erl:183-191",
                 "cases": [["$c", "clientId", "$queue/client/$c", "$queue/client/clientId"],
                           ["${username}", "test", "username/${username}/client/x",
                            "username/test/client/x"],
                           ["${clientid}", "clientId", "username/test/client/${clientid}",
                            "username/test/client/clientId"]]},
    "parse_ok": {"src": "apps/emqx/test/emqx_topic_SUITE.erl:205-213",
                 "cases": [["a/b/+/#", {}, "a/b/+/#", {}],
                           ["a/b/+/#", {"qos": 1}, "a/b/+/#", {"qos": 1}],
                           ["$queue/topic", {}, "topic", {"share": "$queue"}],
                           ["$share/group/topic", {}, "topic", {"share": "group"}],
                           ["$local/topic", {}, "$local/topic", {}],
                           ["$local/$queue/topic", {}, "$local/$queue/topic", {}],
                           ["$local/$share/group/a/b/c", {}, "$local/$share/group/a/b/c", {}],
                           ["$fastlane/topic", {}, "$fastlane/topic", {}]]},
    "parse_err": {"src": "apps/emqx/test/emqx_topic_SUITE.erl:196-204",
                  "cases": [["$queue/t", {"share": "g"}], ["$share/g/t", {"share": "g"}],
                            ["$share/t", {}], ["$share/+/t", {}]]},
}

# emqx_router_SUITE t_match_routes (emqx_router_SUITE.erl:81-95)
ROUTER_CASES = [
    {"name": "t_match_routes", "src": "apps/emqx/test/emqx_router_SUITE.erl:81-95",
     "add": ["a/b/c", "a/+/c", "a/b/#", "#"],
     "queries": [["a/b/c", ["#", "a/+/c", "a/b/#", "a/b/c"]]],
     "then_delete_all": [["a/b/c", []]]},
]

# emqx_client_SUITE: fixed topic sets (:28-43) and the delivery expectations that
# pin match sets: overlapping subscriptions (:165-187) and $-topics (:225-238).
CLIENT = {
    "src": "apps/emqx/test/emqx_client_SUITE.erl:28-43,165-187,225-238",
    "TOPICS": ["TopicA", "TopicA/B", "Topic/C", "TopicA/C", "/TopicA"],
    "WILD_TOPICS": ["TopicA/+", "+/C", "#", "/#", "/+", "+/+", "TopicA/#"],
    # t_overlapping_subscriptions: subs {TopicA/#, TopicA/+}, publish TopicA/C -> both filters match
    "overlapping": {"subs": ["TopicA/#", "TopicA/+"], "topic": "TopicA/C",
                    "expect": ["TopicA/#", "TopicA/+"]},
    # t_dollar_topics: sub '+/+', publish '$TopicA/B' -> no delivery
    "dollar": {"subs": ["+/+"], "topic": "$TopicA/B", "expect": []},
}

# emqx_broker_bench run1 (apps/emqx/src/emqx_broker_bench.erl:25-34,161-162):
# every publisher topic matches exactly one route.
BENCH = {"src": "apps/emqx/src/emqx_broker_bench.erl:25-34,146-162",
         "subscribers": 80, "sub_ops": 1000, "publishers": 80,
         "sub_ptn": "device/{{id}}/+/{{num}}/#",
         "pub_ptn": "device/{{id}}/foo/{{num}}/bar/1/2/3/4/5",
         "expect_routes_per_topic": 1}


# emqx_retainer_SUITE (mnesia backend): retained topics as stored, then the subscriptions a
# client makes and the messages it receives.  ops: ["store", topic, expiry_ms] (0 = never,
# emqx_retainer.erl:157-168 with msg_expiry_interval "0s"), ["publish_empty", topic] (a
# retained empty payload deletes, emqx_retainer.erl:90-101), ["delete", topic]
# (emqx_retainer:delete/1 -> delete_message/2, wildcard -> match_delete_messages/1).
# queries: [now_ms, filter, expected sorted topics] — dispatch/4 picks read_message/2 for a
# plain filter (expiry >= now) and match_messages/3 for a wildcard one (expiry > now).
T0 = 1_000_000
RETAIN_CASES = [
    {"name": "t_wildcard_subscription", "src": "apps/emqx_retainer/test/emqx_retainer_SUITE.erl:154-177",
     "ops": [["store", "retained/0", 0], ["store", "retained/1", 0], ["store", "retained/a/b/c", 0]],
     "queries": [[T0, "retained/+", ["retained/0", "retained/1"]],
                 [T0, "retained/+/b/#", ["retained/a/b/c"]]]},
    {"name": "t_message_expiry", "src": "apps/emqx_retainer/test/emqx_retainer_SUITE.erl:179-221",
     "ops": [["store", "retained/0", 0], ["store", "retained/1", T0 + 2000], ["store", "retained/2", T0 + 5000],
             ["store", "retained/3", 0], ["store", "$SYS/retained/4", 0]],
     "queries": [[T0, "retained/+", ["retained/0", "retained/1", "retained/2", "retained/3"]],
                 [T0, "$SYS/retained/+", ["$SYS/retained/4"]],
                 [T0 + 3000, "retained/+", ["retained/0", "retained/2", "retained/3"]],
                 [T0 + 3000, "$SYS/retained/+", ["$SYS/retained/4"]]]},
    {"name": "t_message_expiry_2", "src": "apps/emqx_retainer/test/emqx_retainer_SUITE.erl:223-238",
     "ops": [["store", "retained", T0 + 2000]],
     "queries": [[T0, "retained", ["retained"]], [T0 + 4000, "retained", []]]},
    {"name": "t_clean", "src": "apps/emqx_retainer/test/emqx_retainer_SUITE.erl:240-263",
     "ops": [["store", "retained/0", 0], ["store", "retained/1", 0], ["store", "retained/test/0", 0]],
     "queries": [[T0, "retained/#", ["retained/0", "retained/1", "retained/test/0"]]],
     "then": [["delete", "retained/test/0"], ["delete", "retained/+"]],
     "after": [[T0, "retained/#", []]]},
    {"name": "t_retain_handling", "src": "apps/emqx_retainer/test/emqx_retainer_SUITE.erl:110-152",
     "ops": [],
     "queries": [[T0, "retained", []], [T0, "retained/#", []]],
     "then": [["store", "retained", 0]],
     "after": [[T0, "retained", ["retained"]], [T0, "retained/#", ["retained"]]]},
    {"name": "t_store_and_clean_empty_payload", "src": "apps/emqx_retainer/test/emqx_retainer_SUITE.erl:89-108",
     "ops": [["store", "retained", 0]],
     "queries": [[T0, "retained", ["retained"]]],
     "then": [["publish_empty", "retained"]],
     "after": [[T0, "retained", []]]},
    {"name": "t_flow_control_set", "src": "apps/emqx_retainer/test/emqx_retainer_SUITE.erl:284-310",
     "ops": [["store", "retained/0", 0], ["store", "retained/1", 0], ["store", "retained/3", 0]],
     "queries": [[T0, "retained/#", ["retained/0", "retained/1", "retained/3"]]]},
]


def main():
    out = {
        "generated_by": "tests/golden/make_kats.py",
        "reference": "xiongzhenhai-zh/emqx @ EMQX 5.0.0-beta.3",
        "trie_cases": TRIE_CASES,
        "eunit": EUNIT,
        "topic_match": TOPIC_MATCH,
        "topic_misc": TOPIC_MISC,
        "router_cases": ROUTER_CASES,
        "client": CLIENT,
        "bench": BENCH,
        "retain_cases": RETAIN_CASES,
    }
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "kats.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
        f.write("\n")
    print("wrote", path)


if __name__ == "__main__":
    main()

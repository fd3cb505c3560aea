#!/usr/bin/env python3
"""Per-iteration kernel breakdown of a PPO_AcM bench run from a rocprofv3 kernel trace.

usage: ppo_breakdown.py <run_kernel_trace.csv> <warmup iterations> <timed iterations>

The window is K whole iterations: from the GAE launch of iteration `warmup` (one k_gae_* launch per
iteration) to the GAE launch of iteration warmup + K.  Every kernel starting inside it is put in a
category (rollout / critic / actor / ACM / GAE / obs statistics / other) and summed; `busy` is the union
of the kernel intervals (two streams overlap: the ACM epochs run beside the critic / actor update), and
`span` the window's wall time on the device.  All figures are ms per iteration.
"""
import csv
import sys
from collections import defaultdict


def category(name):
    n = name.split("(")[0]
    if "k_mlp_sgd<" in n:
        inner = n.split("k_mlp_sgd<")[1]
        head = inner.split(",")[3].strip().rstrip(">")
        return {"0": "acm epoch (k_mlp_sgd HEAD 0)", "1": "actor epoch (k_mlp_sgd HEAD 1)",
                "2": "critic steps (k_mlp_sgd HEAD 2)"}.get(head, "k_mlp_sgd ?")
    if "k_gae" in n:
        return "gae"
    if any(k in n for k in ("k_onp_critic", "k_onp_finish_critic")):
        return "critic per-step path"
    if any(k in n for k in ("k_onp_actor", "k_onp_finish_actor", "k_ppo", "k_adv")):
        return "actor per-step path"
    if "k_onp_value" in n:
        return "critic value"
    if "k_dw" in n:
        return "dW (per-step paths)"
    if "k_adam" in n:
        return "adam (per-step paths)"
    if any(k in n for k in ("k_onp_act", "k_policy_act", "k_synth", "k_episode", "k_rand", "k_replay_add")):
        return "rollout"
    if "k_st_" in n or "stats" in n:
        return "obs statistics"
    if "rocprim" in n or "k_perm" in n or "sort" in n.lower():
        return "permutations"
    return "other: " + n[:60]


def main():
    path, warm, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    rows = list(csv.DictReader(open(path)))
    iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                 r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rows)
    gae = [x[0] for x in iv if "k_gae" in x[2]]
    if len(gae) < warm + K + 1:
        K = len(gae) - warm - 1
    t0, t1 = gae[warm], gae[warm + K]
    win = [x for x in iv if t0 <= x[0] < t1]
    cat = defaultdict(lambda: [0, 0.0])
    for s, e, n, _ in win:
        c = cat[category(n)]
        c[0] += 1
        c[1] += (e - s) * 1e-6

    def union(xs):
        tot, cur_s, cur_e = 0.0, None, None
        for s, e in sorted(xs):
            if cur_e is None or s > cur_e:
                if cur_e is not None:
                    tot += cur_e - cur_s
                cur_s, cur_e = s, e
            else:
                cur_e = max(cur_e, e)
        if cur_e is not None:
            tot += cur_e - cur_s
        return tot * 1e-6

    busy = union([(s, min(e, t1)) for s, e, _, _ in win])
    print("window: %d iterations, span %.3f ms/iter, device busy (union) %.3f ms/iter" % (K, (t1 - t0) * 1e-6 / K,
                                                                                         busy / K))
    qs = defaultdict(list)
    for s, e, _, q in win:
        qs[q].append((s, min(e, t1)))
    for q, xs in sorted(qs.items()):
        print("  queue %s: busy %.3f ms/iter over %d launches" % (q, union(xs) / K, len(xs)))
    print("%-40s %9s %12s" % ("category", "launches", "ms/iter"))
    for k, (c, ms) in sorted(cat.items(), key=lambda kv: -kv[1][1]):
        print("%-40s %9.1f %12.3f" % (k, c / K, ms / K))


if __name__ == "__main__":
    main()

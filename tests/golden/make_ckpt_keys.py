"""Key structure of the reference's shipped checkpoints (/root/reference/models/*.pkl) ->
tests/golden/ref_ckpt_keys.json.

The checkpoints are pickles whose tensors need torch.storage._load_from_bytes; torch's weights-only
unpickler refuses them (protocol-3 BINBYTES opcode), so they are never LOADED here.  This script only
DISASSEMBLES the opcode stream with pickletools.genops (no object is constructed, no global is
resolved) and keeps the string constants, from which the nested key order of the reference's
collect_params_dict / state_dict (rltoolkit/rl.py:263-301, algorithms/sac/sac.py:287-309,
acm/off_policy/ddpg_acm.py:87-94) is read: top-level keys, and each network's parameter names in
state_dict order.  Run in this container (needs /root/reference):  python tests/golden/make_ckpt_keys.py
"""
import json
import os
import pickletools

SRC = "/root/reference/models"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ref_ckpt_keys.json")
TOP = ("actor", "critic", "critic_1", "critic_2", "acm", "obs_mean", "obs_std", "min_obs", "max_obs")
PARAM_NO_DOT = ("t", "t1", "log_scale")
STR_OPS = ("BINUNICODE", "SHORT_BINUNICODE", "BINUNICODE8", "UNICODE", "SHORT_BINSTRING", "BINSTRING")


def keys_of(path):
    with open(path, "rb") as f:
        data = f.read()
    strs = [arg for op, arg, _ in pickletools.genops(data) if op.name in STR_OPS]
    out, cur = {}, None
    for s in strs:
        if s in TOP and (cur is None or s not in out):
            out[s] = []
            cur = s
        elif cur is not None and ("." in s or s in PARAM_NO_DOT):
            out[cur].append(s)
    return {k: (v if v else None) for k, v in out.items()}  # None: a plain tensor entry


def main():
    res = {}
    for fn in sorted(os.listdir(SRC)):
        if fn.endswith(".pkl"):
            res[fn] = keys_of(os.path.join(SRC, fn))
    with open(OUT, "w") as f:
        json.dump(res, f, indent=1)
    print("wrote", OUT, list(res))


if __name__ == "__main__":
    main()

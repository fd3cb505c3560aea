"""Checkpoints in the reference's format (rltoolkit/rl.py:281-301): a pickle of the
``collect_params_dict`` dict -- per network an OrderedDict state_dict of CPU fp32 tensors
(keys in the reference's state_dict order), plus obs_mean / obs_std / min_obs / max_obs.  A
checkpoint written here loads in the reference with its own ``pkl.load`` and vice versa in
structure (tests/test_checkpoint.py pins the key structure against the reference's shipped
models, tests/golden/ref_ckpt_keys.json).

Loading never executes code from the file: torch's weights-only loader for torch zip files, and
for plain pickles a restricted unpickler that resolves only the constructors a state-dict pickle
needs (OrderedDict, torch's tensor rebuild, storage-from-bytes routed through
``torch.load(weights_only=True)``); any other global is refused.
"""
import collections
import io
import pickle
import zipfile

import torch


def _state(sd):
    return collections.OrderedDict((k, torch.as_tensor(v).detach().cpu().clone()) for k, v in sd.items())


def save_params(path, params):
    """pickle.dump of {name: OrderedDict state_dict | tensor | None} (rl.py:286-292)."""
    out = {}
    for k, v in params.items():
        out[k] = _state(v) if isinstance(v, dict) else (None if v is None else torch.as_tensor(v).cpu())
    with open(path, "wb") as f:
        pickle.dump(out, f)


def _storage_from_bytes(b):
    return torch.load(io.BytesIO(b), weights_only=True)


class _StateDictUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ("collections", "OrderedDict"): collections.OrderedDict,
        ("torch._utils", "_rebuild_tensor_v2"): torch._utils._rebuild_tensor_v2,
        ("torch.storage", "_load_from_bytes"): _storage_from_bytes,
    }

    def find_class(self, module, name):
        fn = self._ALLOWED.get((module, name))
        if fn is None:
            raise pickle.UnpicklingError("checkpoint refers to %s.%s: not a state-dict pickle" % (module, name))
        return fn


def load_params(path):
    """The dict written by save_params (or by the reference's save)."""
    if zipfile.is_zipfile(path):
        return torch.load(path, weights_only=True, map_location="cpu")
    with open(path, "rb") as f:
        return _StateDictUnpickler(f).load()

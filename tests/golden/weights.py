"""Deterministic parameter fill shared by the golden generator and the tests.

Golden fixtures do not store initial weights: both sides rebuild them from a
numpy seed with this helper, iterating a ``state_dict``-ordered list of
(name, shape) pairs.  Weights/biases follow nn.Linear's U(-1/sqrt(fan_in), +)
range so activations stay in the same regime as the reference's own init.
"""
import numpy as np


def fill_params(named_shapes, seed):
    """named_shapes: iterable of (name, shape). Returns {name: float32 array}."""
    rng = np.random.RandomState(seed)
    out = {}
    fan_in = None
    for name, shape in named_shapes:
        shape = tuple(shape)
        if name.endswith("weight") and len(shape) == 2:
            fan_in = shape[1]
            k = 1.0 / np.sqrt(fan_in)
        elif fan_in is not None:
            k = 1.0 / np.sqrt(fan_in)
        else:
            k = 0.5
        if name in ("t", "t1"):  # BasicAcM scale parameters
            out[name] = (1.0 + 0.1 * rng.uniform(-1, 1, size=shape)).astype(np.float32)
        else:
            out[name] = rng.uniform(-k, k, size=shape).astype(np.float32)
    return out

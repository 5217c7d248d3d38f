"""Parameter specs (state_dict key order and shapes) and deterministic initialisers.

The key names and their order are the reference's ``nn.Module.state_dict()`` order, so
checkpoints written by this package load into the reference and vice versa:

* ``Connect4Net``   -- connect4/Connect4Net.py:18-25
* ``TicTacToeNet``  -- tictactoe/TicTacToeNet.py:16-26
* ``PolicyValueGNN``-- gnn_utils.py:5-28 (GNNLayer) and :93-105 (output_transform)

Two initialisers exist:

* :func:`torch_default_init` reproduces ``nn.Linear``/``nn.Conv2d`` default init
  (kaiming_uniform(a=sqrt(5)) -> U(-1/sqrt(fan_in), 1/sqrt(fan_in)) for weight then bias,
  module by module) on the torch CPU generator, i.e. the exact values the reference gets
  from the same ``torch.manual_seed``.
* :func:`synthetic_state_dict` is the documented PCG64 generator used for the 479 MB
  Connect4 GNN weights in the goldens, which are never committed.
"""
from collections import OrderedDict
import math

import numpy as np


def connect4_net_spec(n=7, action_size=None):
    """connect4/Connect4Net.py:18-25 (board n x n, A = n + 1, Connect4Game.py:139-141)."""
    a = n + 1 if action_size is None else action_size
    f = 64 * n * n
    return [
        ("conv1.weight", (32, 1, 3, 3)), ("conv1.bias", (32,)),
        ("conv2.weight", (64, 32, 3, 3)), ("conv2.bias", (64,)),
        ("fc_policy.weight", (a, f)), ("fc_policy.bias", (a,)),
        ("fc_value.weight", (1, f)), ("fc_value.bias", (1,)),
    ]


def tictactoe_net_spec(n=3, action_size=None):
    """tictactoe/TicTacToeNet.py:16-26 (A = n*n + 1, TicTacToeGame.py:392-394)."""
    a = n * n + 1 if action_size is None else action_size
    f = 128 * (n - 2) * (n - 2)
    return [
        ("conv1.weight", (32, 1, 3, 3)), ("conv1.bias", (32,)),
        ("conv2.weight", (64, 32, 3, 3)), ("conv2.bias", (64,)),
        ("conv3.weight", (128, 64, 3, 3)), ("conv3.bias", (128,)),
        ("fc1.weight", (512, f)), ("fc1.bias", (512,)),
        ("fc_policy.weight", (a, 512)), ("fc_policy.bias", (a,)),
        ("fc2.weight", (512, f)), ("fc2.bias", (512,)),
        ("fc_value.weight", (1, 512)), ("fc_value.bias", (1,)),
    ]


def gnn_spec(feature_dim, num_layers=2, hidden=128):
    """gnn_utils.py:11-28 per layer, then output_transform gnn_utils.py:101-105."""
    f = feature_dim
    spec = []
    for i in range(num_layers):
        p = f"layers.{i}."
        spec += [
            (p + "attention.0.weight", (hidden, 2 * f)), (p + "attention.0.bias", (hidden,)),
            (p + "attention.2.weight", (1, hidden)), (p + "attention.2.bias", (1,)),
            (p + "update_net.0.weight", (f, 2 * f)), (p + "update_net.0.bias", (f,)),
            (p + "update_net.2.weight", (f, f)), (p + "update_net.2.bias", (f,)),
            (p + "gate.0.weight", (f, 2 * f)), (p + "gate.0.bias", (f,)),
        ]
    spec += [
        ("output_transform.0.weight", (f, f)), ("output_transform.0.bias", (f,)),
        ("output_transform.2.weight", (f, f)), ("output_transform.2.bias", (f,)),
    ]
    return spec


def spec_numel(spec):
    return sum(int(np.prod(s)) for _, s in spec)


def _fan_in(spec):
    """fan_in per key: a bias uses the fan_in of the weight declared just before it."""
    out, last = {}, None
    for k, s in spec:
        if k.endswith("weight"):
            last = int(np.prod(s[1:]))
        out[k] = last
    return out


def synthetic_state_dict(spec, seed):
    """PCG64(seed) stream, tensor by tensor in spec order:
    ``w = (2*u - 1) * (1/sqrt(fan_in))`` with ``u = rng.random(shape, float32)``, all float32.
    """
    rng = np.random.Generator(np.random.PCG64(seed))
    fans = _fan_in(spec)
    sd = OrderedDict()
    for k, s in spec:
        bound = np.float32(1.0 / math.sqrt(fans[k]))
        u = rng.random(s, dtype=np.float32)
        sd[k] = ((u * np.float32(2.0) - np.float32(1.0)) * bound).astype(np.float32)
    return sd


def torch_default_init(spec, generator=None):
    """Same values as constructing the reference modules under the same torch seed:
    each module draws ``weight.uniform_(-b, b)`` then ``bias.uniform_(-b, b)`` in
    declaration order with b = 1/sqrt(fan_in) (torch.nn.Linear.reset_parameters)."""
    import torch
    fans = _fan_in(spec)
    sd = OrderedDict()
    for k, s in spec:
        t = torch.empty(s, dtype=torch.float32)
        if k.endswith("weight"):
            # kaiming_uniform_(a=sqrt(5)): gain = sqrt(2/(1+5)), bound = gain*sqrt(3/fan_in)
            gain = math.sqrt(2.0 / (1 + 5))
            bound = gain * math.sqrt(3.0 / fans[k])
        else:
            bound = 1.0 / math.sqrt(fans[k]) if fans[k] > 0 else 0.0
        with torch.no_grad():
            t.uniform_(-bound, bound, generator=generator)
        sd[k] = t
    return sd

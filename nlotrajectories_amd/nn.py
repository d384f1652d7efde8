"""Learned-SDF models and their flattened weights.

`FourierMLP` / `SIREN` restate the reference architectures (core/nn_architectures.py:8-100) as
torch modules so users can train or load them; `MultiLayerPerceptron` restates l4casadi's naive
MLP used for `model.type: mlp` (scripts/run_benchmark.py:64-65; external l4casadi, unpinned:
Linear(in,H) -> act -> (hidden_layers - 1) x [Linear(H,H) -> act] -> Linear(H,out), SURVEY.md §8a a5;
`hidden_layers` counts the hidden activations, so the YAMLs' num_hidden_layers: 2 is ONE HxH layer).

`MlpWeights` is the flat fp32 form the HIP kernel consumes (NlotMlpDesc in include/nlot.h).
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Dict

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from . import _abi

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
ARTEFACT_NPZ = os.path.join(DATA_DIR, "nn_sdf_artefact.npz")


class FourierFeatureLayer(nn.Module):
    """cos(x @ W + b) * scale, core/nn_architectures.py:30-38."""

    def __init__(self, in_features, out_features, scale=1.0):
        super().__init__()
        self.scale = scale
        self.weights = nn.Parameter(torch.randn(in_features, out_features) * scale)
        self.bias = nn.Parameter(torch.zeros(out_features))

    def forward(self, x):
        return torch.cos(x @ self.weights + self.bias) * self.scale


class FourierMLP(nn.Module):
    """core/nn_architectures.py:42-72 (num_layers-2 hidden Linear+act layers)."""

    _ACTS = {"ReLU": F.relu, "tanh": torch.tanh, "sigmoid": torch.sigmoid, "leaky_relu": F.leaky_relu}

    def __init__(self, input_dim, hidden_dim, output_dim, num_layers=3, scale=1.0, activation_function="ReLU"):
        super().__init__()
        if activation_function not in self._ACTS:
            raise ValueError(f"Unsupported activation function: {activation_function}")
        self.activation_name = activation_function
        self.activation_function = self._ACTS[activation_function]
        self.fourier = FourierFeatureLayer(input_dim, hidden_dim, scale)
        self.layers = nn.ModuleList([nn.Linear(hidden_dim, hidden_dim) for _ in range(num_layers - 2)])
        self.output_layer = nn.Linear(hidden_dim, output_dim)

    def forward(self, x):
        x = self.fourier(x)
        for layer in self.layers:
            x = self.activation_function(layer(x))
        return self.output_layer(x)


class MultiLayerPerceptron(nn.Module):
    """l4casadi.naive.MultiLayerPerceptron(in, hidden, out, hidden_layers, activation) restated.

    `hidden_layers` hidden activations: input Linear(in, H), then hidden_layers - 1 Linear(H, H), then
    Linear(H, out) (l4casadi is external and unpinned, so the layer count is the
    survey's record of its source).  The ReLU kernels consume it through MlpWeights.from_module."""

    _ACTS = {"ReLU": F.relu, "Tanh": torch.tanh, "Sigmoid": torch.sigmoid, "LeakyReLU": F.leaky_relu,
             None: lambda x: x}

    def __init__(self, in_features, hidden_features, out_features, hidden_layers, activation=None):
        super().__init__()
        if hidden_layers < 1:
            raise ValueError("There must be at least one hidden layer")
        if activation not in self._ACTS:
            raise ValueError(f"Unsupported activation: {activation}")
        self.input_layer = nn.Linear(in_features, hidden_features)
        self.hidden_layers = nn.ModuleList([nn.Linear(hidden_features, hidden_features)
                                            for _ in range(hidden_layers - 1)])
        self.output_layer = nn.Linear(hidden_features, out_features)
        self.activation = activation
        self.act = self._ACTS[activation]

    def forward(self, x):
        x = self.act(self.input_layer(x))
        for layer in self.hidden_layers:
            x = self.act(layer(x))
        return self.output_layer(x)


class SineLayer(nn.Module):
    """core/nn_architectures.py:8-26."""

    def __init__(self, in_features, out_features, bias=True, is_first=False, omega_0=30):
        super().__init__()
        self.omega_0, self.is_first = omega_0, is_first
        self.linear = nn.Linear(in_features, out_features, bias=bias)
        with torch.no_grad():
            if is_first:
                self.linear.weight.uniform_(-1 / in_features, 1 / in_features)
            else:
                b = math.sqrt(6 / in_features) / omega_0
                self.linear.weight.uniform_(-b, b)

    def forward(self, x):
        return torch.sin(self.omega_0 * self.linear(x))


class SIREN(nn.Module):
    """core/nn_architectures.py:75-100 (the SDF kernels take it as in_kind LINEAR + NLOT_ACT_SINE)."""

    def __init__(self, input_dim, hidden_dim, output_dim, num_layers=3, omega_0=30):
        super().__init__()
        self.layers = nn.ModuleList([SineLayer(input_dim, hidden_dim, is_first=True, omega_0=omega_0)])
        for _ in range(num_layers - 2):
            self.layers.append(SineLayer(hidden_dim, hidden_dim, omega_0=omega_0))
        self.output_layer = nn.Linear(hidden_dim, output_dim)

    def forward(self, x):
        for layer in self.layers:
            x = layer(x)
        return self.output_layer(x)


# activation codes <-> the reference's names (FourierMLP: nn_architectures.py:47-52; naive MLP: l4casadi)
_FOURIER_ACT_NAMES = {_abi.ACT_RELU: "ReLU", _abi.ACT_TANH: "tanh", _abi.ACT_SIGMOID: "sigmoid",
                      _abi.ACT_LEAKY_RELU: "leaky_relu"}
_NAIVE_ACT_NAMES = {_abi.ACT_RELU: "ReLU", _abi.ACT_TANH: "Tanh", _abi.ACT_SIGMOID: "Sigmoid",
                    _abi.ACT_LEAKY_RELU: "LeakyReLU"}


@dataclass
class MlpWeights:
    """Flat fp32 weights: h0 = phi(p @ A + b0); n_hidden x relu(W h + b); f = w_out . h + b_out."""

    in_kind: int
    hidden: int
    n_hidden: int
    fourier_scale: float  # FourierFeatureLayer.scale; omega_0 for SIREN (act = ACT_SINE)
    b_out: float
    arrays: Dict[str, np.ndarray]
    act: int = _abi.ACT_RELU  # hidden activation (and the input layer's, in_kind LINEAR)

    @property
    def flops_per_point_fwd(self) -> int:
        H = self.hidden
        return 2 * (2 * H + self.n_hidden * H * H + H)

    @property
    def flops_per_point_fwd_grad(self) -> int:
        return 2 * self.flops_per_point_fwd

    def to(self, dtype=np.float32):
        return self

    def torch_module(self) -> nn.Module:
        """Equivalent torch module (fp32), for reference evaluation in tests / the numpy path."""
        H = self.hidden
        if self.act == _abi.ACT_SINE and self.in_kind != _abi.MLP_IN_FOURIER:
            m = SIREN(2, H, 1, num_layers=self.n_hidden + 2, omega_0=self.fourier_scale)
            sd = {"layers.0.linear.weight": self.arrays["A"].T, "layers.0.linear.bias": self.arrays["b0"]}
            for l in range(self.n_hidden):
                sd[f"layers.{l + 1}.linear.weight"] = self.arrays["W"][l]
                sd[f"layers.{l + 1}.linear.bias"] = self.arrays["b"][l]
        elif self.in_kind == _abi.MLP_IN_FOURIER:
            m = FourierMLP(2, H, 1, num_layers=self.n_hidden + 2, scale=self.fourier_scale,
                           activation_function=_FOURIER_ACT_NAMES[self.act])
            sd = {"fourier.weights": self.arrays["A"], "fourier.bias": self.arrays["b0"]}
            for l in range(self.n_hidden):
                sd[f"layers.{l}.weight"] = self.arrays["W"][l]
                sd[f"layers.{l}.bias"] = self.arrays["b"][l]
        else:
            m = MultiLayerPerceptron(2, H, 1, self.n_hidden + 1, _NAIVE_ACT_NAMES[self.act])
            sd = {"input_layer.weight": self.arrays["A"].T, "input_layer.bias": self.arrays["b0"]}
            for l in range(self.n_hidden):
                sd[f"hidden_layers.{l}.weight"] = self.arrays["W"][l]
                sd[f"hidden_layers.{l}.bias"] = self.arrays["b"][l]
        sd["output_layer.weight"] = self.arrays["w_out"][None, :]
        sd["output_layer.bias"] = np.array([self.b_out], np.float32)
        m.load_state_dict({k: torch.as_tensor(np.ascontiguousarray(v)) for k, v in sd.items()})
        return m.eval()

    @staticmethod
    def from_module(model: nn.Module) -> "MlpWeights":
        """Flatten a FourierMLP / MultiLayerPerceptron / SIREN into kernel form."""
        g = lambda t: t.detach().cpu().float().numpy().copy()
        if isinstance(model, SIREN):
            first, rest = model.layers[0], list(model.layers[1:])
            H = first.linear.weight.shape[0]
            if first.linear.bias is None or any(l.linear.bias is None for l in rest):
                raise ValueError("SIREN layers without bias are not supported")
            omegas = {float(l.omega_0) for l in model.layers}
            if len(omegas) != 1:
                raise ValueError("SIREN layers must share omega_0")
            arrays = dict(A=g(first.linear.weight).T.copy(), b0=g(first.linear.bias),
                          W=np.stack([g(l.linear.weight) for l in rest]) if rest else np.zeros((0, H, H), np.float32),
                          b=np.stack([g(l.linear.bias) for l in rest]) if rest else np.zeros((0, H), np.float32),
                          w_out=g(model.output_layer.weight)[0])
            return MlpWeights(_abi.MLP_IN_LINEAR_RELU, H, len(rest), omegas.pop(),
                              float(g(model.output_layer.bias)[0]), arrays, _abi.ACT_SINE)
        if isinstance(model, FourierMLP) or hasattr(model, "fourier"):
            act = {v: k for k, v in _FOURIER_ACT_NAMES.items()}[getattr(model, "activation_name", "ReLU")]
            H = model.fourier.weights.shape[1]
            Ws = [g(l.weight) for l in model.layers]
            bs = [g(l.bias) for l in model.layers]
            arrays = dict(A=g(model.fourier.weights), b0=g(model.fourier.bias),
                          W=np.stack(Ws) if Ws else np.zeros((0, H, H), np.float32),
                          b=np.stack(bs) if bs else np.zeros((0, H), np.float32),
                          w_out=g(model.output_layer.weight)[0])
            return MlpWeights(_abi.MLP_IN_FOURIER, H, len(Ws), float(model.fourier.scale),
                              float(g(model.output_layer.bias)[0]), arrays, act)
        if hasattr(model, "input_layer") and hasattr(model, "hidden_layers"):
            name = getattr(model, "activation", "ReLU")
            if name not in _NAIVE_ACT_NAMES.values() or name is None:
                raise ValueError(f"unsupported activation {name!r} for the SDF kernels (DESIGN.md §7)")
            act = {v: k for k, v in _NAIVE_ACT_NAMES.items()}[name]
            H = model.input_layer.weight.shape[0]
            Ws = [g(l.weight) for l in model.hidden_layers]
            bs = [g(l.bias) for l in model.hidden_layers]
            arrays = dict(A=g(model.input_layer.weight).T.copy(), b0=g(model.input_layer.bias),
                          W=np.stack(Ws) if Ws else np.zeros((0, H, H), np.float32),
                          b=np.stack(bs) if bs else np.zeros((0, H), np.float32),
                          w_out=g(model.output_layer.weight)[0])
            return MlpWeights(_abi.MLP_IN_LINEAR_RELU, H, len(Ws), 1.0, float(g(model.output_layer.bias)[0]), arrays,
                              act)
        raise TypeError(f"unsupported model type {type(model).__name__} (DESIGN.md §7)")

    def save(self, path) -> None:
        """Plain npz (no pickle): the arrays plus the scalar fields."""
        np.savez(path, in_kind=self.in_kind, hidden=self.hidden, n_hidden=self.n_hidden,
                 fourier_scale=self.fourier_scale, b_out=self.b_out, act=self.act, **self.arrays)

    @staticmethod
    def load(path) -> "MlpWeights":
        z = np.load(path, allow_pickle=False)
        arrays = {k: z[k].astype(np.float32) for k in ("A", "b0", "W", "b", "w_out")}
        return MlpWeights(int(z["in_kind"]), int(z["hidden"]), int(z["n_hidden"]), float(z["fourier_scale"]),
                          float(z["b_out"]), arrays, int(z["act"]) if "act" in z.files else _abi.ACT_RELU)

    @staticmethod
    def artefact() -> "MlpWeights":
        """The reference artefact _l4c_generated/nn_sdf.pt (FourierMLP 2-128-128-1, scale 10),
        extracted as raw data by tests/golden/make_golden.py."""
        z = np.load(ARTEFACT_NPZ, allow_pickle=False)
        H = z["A"].shape[1]
        arrays = dict(A=z["A"].astype(np.float32), b0=z["b0"].astype(np.float32),
                      W=z["W1"].astype(np.float32)[None], b=z["b1"].astype(np.float32)[None],
                      w_out=z["w2"].astype(np.float32)[0])
        return MlpWeights(_abi.MLP_IN_FOURIER, H, 1, float(z["scale"]), float(z["b2"][0]), arrays)

    @staticmethod
    def random_relu_mlp(hidden=256, n_hidden=3, seed=0) -> "MlpWeights":
        """Seeded kaiming-uniform ReLU MLP with n_hidden HxH layers (the stress config 2-256x4-1 is
        n_hidden = 3: four hidden activations; init as core/sdf/l4casadi.py:69-74)."""
        gen = torch.Generator().manual_seed(seed)
        m = MultiLayerPerceptron(2, hidden, 1, n_hidden + 1, "ReLU")
        with torch.no_grad():
            for mod in m.modules():
                if isinstance(mod, nn.Linear):
                    bound = math.sqrt(6.0 / mod.weight.shape[1])
                    mod.weight.uniform_(-bound, bound, generator=gen)
                    mod.bias.zero_()
        return MlpWeights.from_module(m)

    @staticmethod
    def stress_sdf_mlp(seed=0, hidden=256, n_hidden=3) -> "MlpWeights":
        """The stress configuration's SDF net: random_relu_mlp(256, 3, seed) with its output bias set to
        minus the median of the net over a 64 x 64 grid of the sampling box [-0.3, 1.3]^2, so that about
        half of the box is free space (a zero-bias ReLU net is positively homogeneous, and seed 0 is
        negative on 98 % of the box)."""
        w = MlpWeights.random_relu_mlp(hidden, n_hidden, seed)
        m = w.torch_module().double()
        g = torch.linspace(-0.3, 1.3, 64, dtype=torch.float64)
        P = torch.stack(torch.meshgrid(g, g, indexing="ij"), -1).reshape(-1, 2)
        with torch.no_grad():
            med = m(P)[:, 0].median().item()
            m.output_layer.bias.fill_(-med)
        return MlpWeights.from_module(m.float())

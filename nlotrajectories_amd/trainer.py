"""Learned-SDF production: the reference's `sample_points` / `NNObstacleTrainer` (core/sdf/l4casadi.py:14-228)
restated on PyTorch-ROCm, seeded.

The reference trains one network per run in l4casadi mode (scripts/run_benchmark.py:84-95): targets are the
scene's exact SDF (`MultiObstacle.sdf` = min of the obstacles' exact SDFs, shapely for polygons; here
`scene.exact_sdf`), the loss is MSE + surface loss (core/metrics.py:83-110) + eikonal loss, optimised by Adam
with early stopping on a 10 % validation split.  Differences, all deliberate:

* seeded: numpy's `default_rng(seed)` replaces the global `np.random` of `sample_points`, a `torch.Generator`
  the global torch RNG of `randperm` / the shuffling DataLoader / `initialize_weights`;
* the batches come from a device-resident permutation instead of a DataLoader (same batch size, same
  shuffling per epoch, no host round trips);
* `generate_data` passes `boundary_fraction` into `sample_points`' `margin` slot, as the reference does
  (l4casadi.py:118), so the band around the boundary is |sdf| < boundary_fraction while the boundary share of
  the samples stays at the default 0.3 — reproduced, not fixed.

The product consumes the trained module through `MlpWeights.from_module` (ReLU MLP / FourierMLP kernels).
"""
from __future__ import annotations

import copy

import numpy as np
import torch
import torch.nn as nn

from . import scene


def sample_points(x_range, y_range, n_samples, sdf=None, margin=0.1, boundary_fraction=0.3, random=True,
                  rng: np.random.Generator = None):
    """core/sdf/l4casadi.py:14-66: n_global uniform (or grid) points, plus up to boundary_fraction x n_samples
    points with |sdf| < margin found by rejection (at most 10 x n_boundary rounds).  `sdf(xs, ys)` is the
    scene's exact SDF on numpy arrays."""
    rng = rng or np.random.default_rng(0)
    n_boundary = int(n_samples * boundary_fraction)
    n_global = n_samples - n_boundary
    if random:
        xs = rng.uniform(*x_range, size=n_global)
        ys = rng.uniform(*y_range, size=n_global)
    else:
        side = int(np.sqrt(n_global))
        xs, ys = np.meshgrid(np.linspace(*x_range, side), np.linspace(*y_range, side))
        xs, ys = xs.ravel(), ys.ravel()
    if sdf is not None and n_boundary > 0:
        bx, by, tries = [], [], 0
        while sum(len(b) for b in bx) < n_boundary and tries < n_boundary * 10:
            xc = rng.uniform(*x_range, size=n_boundary)
            yc = rng.uniform(*y_range, size=n_boundary)
            m = np.abs(sdf(xc, yc)) < margin
            bx.append(xc[m])
            by.append(yc[m])
            tries += 1
        bx = np.concatenate(bx)[:n_boundary] if bx else np.zeros(0)
        by = np.concatenate(by)[:n_boundary] if by else np.zeros(0)
        xs, ys = np.concatenate([xs, bx]), np.concatenate([ys, by])
    return xs, ys


def initialize_weights(model: nn.Module, generator: torch.Generator = None):
    """core/sdf/l4casadi.py:69-74: kaiming-uniform (ReLU gain) weights, zero biases."""
    for layer in model.modules():
        if isinstance(layer, nn.Linear):
            with torch.no_grad():
                fan_in = layer.weight.shape[1]
                bound = np.sqrt(6.0 / fan_in)  # gain sqrt(2) x sqrt(3 / fan_in)
                layer.weight.uniform_(-bound, bound, generator=generator)
                if layer.bias is not None:
                    layer.bias.zero_()


def surface_loss(target: torch.Tensor, pred: torch.Tensor, eps: float = 1e-2):
    """core/metrics.py:83-110 (torch branch): mean pred^2 where |target| < eps, or None."""
    m = target.reshape(-1).abs() < eps
    if not bool(m.any()):
        return None
    return (pred.reshape(-1)[m] ** 2).mean()


class NNObstacleTrainer:
    """core/sdf/l4casadi.py:77-228 with the same constructor arguments (plus `seed`); `obstacles` is the scene
    (a list of obstacle dicts in the YAML vocabulary)."""

    def __init__(self, obstacles, model: nn.Module, device=None, epochs: int = 100, eikonal_weight: float = 0,
                 surface_loss_weight: float = 0, n_samples: int = 200000, boundary_fraction: float = 0.3,
                 random: bool = True, batch_size: int = 256, lr: float = 1e-3, seed: int = 0, verbose: bool = True):
        self.obstacles = obstacles
        if device is None:
            device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
        self.device = torch.device(device)
        self.seed = seed
        self.gen = torch.Generator().manual_seed(seed)
        initialize_weights(model, self.gen)
        self.model = model.to(self.device)
        self.epochs, self.eikonal_weight, self.surface_loss_weight = epochs, eikonal_weight, surface_loss_weight
        self.n_samples, self.boundary_fraction, self.random = n_samples, boundary_fraction, random
        self.batch_size, self.lr, self.verbose = batch_size, lr, verbose
        self.history = []
        if verbose:
            print(f"Using surface loss weight: {surface_loss_weight}, eikonal weight: {eikonal_weight}", flush=True)

    def sdf(self, x, y):
        return scene.exact_sdf(self.obstacles, x, y)

    def generate_data(self, x_range, y_range, n_samples, random=True):
        """l4casadi.py:111-123 (boundary_fraction lands in sample_points' margin slot, as there)."""
        xs, ys = sample_points(x_range, y_range, n_samples, self.sdf, self.boundary_fraction, random=random,
                               rng=np.random.default_rng(self.seed))
        inputs = torch.tensor(np.stack([xs, ys], axis=1), dtype=torch.float32)
        targets = torch.tensor(self.sdf(xs, ys), dtype=torch.float32).unsqueeze(1)
        return inputs, targets

    def _loss(self, xb, yb, loss_fn, surface_loss_eps, train):
        if train and self.eikonal_weight > 0:
            xb = xb.requires_grad_(True)
        pred = self.model(xb)
        loss = loss_fn(pred, yb)
        if self.surface_loss_weight > 0:
            sl = surface_loss(yb, pred, eps=surface_loss_eps)
            if sl is not None:
                loss = loss + self.surface_loss_weight * sl
        if train and self.eikonal_weight > 0:
            (g,) = torch.autograd.grad(pred, xb, grad_outputs=torch.ones_like(pred), create_graph=True,
                                       retain_graph=True, only_inputs=True)
            loss = loss + self.eikonal_weight * ((torch.linalg.norm(g, dim=1) - 1.0) ** 2).mean()
        return loss

    def train(self, x_range, y_range, early_stop=True, patience=10, min_delta=1e-4, surface_loss_eps=1e-2):
        """l4casadi.py:125-228: 90/10 split, Adam, per-epoch validation, early stopping on the validation loss,
        best state restored."""
        X, Y = self.generate_data(x_range, y_range, self.n_samples, self.random)
        idx = torch.randperm(len(X), generator=self.gen)
        X, Y = X[idx].to(self.device), Y[idx].to(self.device)
        n_val = int(0.1 * len(X))
        X_val, Y_val, X_tr, Y_tr = X[:n_val], Y[:n_val], X[n_val:], Y[n_val:]
        opt = torch.optim.Adam(self.model.parameters(), lr=self.lr)
        loss_fn = nn.MSELoss()
        best, best_state, bad = float("inf"), copy.deepcopy(self.model.state_dict()), 0
        bs = self.batch_size
        self.model.train()
        for ep in range(self.epochs):
            perm = torch.randperm(len(X_tr), generator=self.gen).to(self.device)
            total = torch.zeros((), device=self.device)
            for i in range(0, len(X_tr), bs):
                j = perm[i:i + bs]
                xb, yb = X_tr[j], Y_tr[j]
                loss = self._loss(xb, yb, loss_fn, surface_loss_eps, True)
                opt.zero_grad()
                loss.backward()
                opt.step()
                total += loss.detach() * len(j)
            self.model.eval()
            val = torch.zeros((), device=self.device)
            with torch.no_grad():
                for i in range(0, n_val, bs):
                    xb, yb = X_val[i:i + bs], Y_val[i:i + bs]
                    val += self._loss(xb, yb, loss_fn, surface_loss_eps, False) * len(xb)
            self.model.train()
            tr_loss, val_loss = float(total) / len(X_tr), float(val) / max(n_val, 1)
            self.history.append((tr_loss, val_loss))
            if self.verbose:
                print(f"Epoch {ep:3d} - Train loss: {tr_loss:.6f} - Val loss: {val_loss:.6f}", flush=True)
            if early_stop:
                if val_loss + min_delta < best:
                    best, bad, best_state = val_loss, 0, copy.deepcopy(self.model.state_dict())
                else:
                    bad += 1
                    if bad >= patience:
                        if self.verbose:
                            print(f"Early stopping at epoch {ep:3d} (no improvement for {patience} epochs).", flush=True)
                        break
        self.model.load_state_dict(best_state)
        self.model.eval()
        return self.model


def model_from_config(mc):
    """scripts/run_benchmark.py:55-83: the network a YAML's `model:` section describes (mlp / fourier / siren)."""
    from .nn import SIREN, FourierMLP, MultiLayerPerceptron

    if mc.type == "mlp":
        return MultiLayerPerceptron(2, mc.hidden_dim, 1, mc.num_hidden_layers, mc.activation_function)
    if mc.type == "fourier":
        return FourierMLP(2, mc.hidden_dim, 1, num_layers=mc.num_hidden_layers + 2,
                          activation_function=mc.activation_function)
    if mc.type == "siren":
        return SIREN(2, mc.hidden_dim, 1, num_layers=mc.num_hidden_layers + 2, omega_0=mc.omega_0)
    raise ValueError(f"Unsupported model type: {mc.type}")


def train_for_config(cfg, seed=0, device=None, epochs=100, verbose=True):
    """run_benchmark.py:84-95: train the config's network on its scene over (-0.5, 1.5)^2."""
    mc = cfg.model
    model = model_from_config(mc)
    tr = NNObstacleTrainer(cfg.obstacle_dicts(), model, device=device, epochs=epochs, n_samples=mc.n_samples,
                           boundary_fraction=mc.boundary_fraction, eikonal_weight=mc.eikonal_loss_weight,
                           surface_loss_weight=mc.surface_loss_weight, seed=seed, verbose=verbose)
    return tr.train((-0.5, 1.5), (-0.5, 1.5)), tr

"""The run-benchmark YAML schema (the reference's core/config.py:26-222, same fields and defaults),
validated with pydantic, and its mapping onto `problem.Problem`.

Sections: `body` (shape, dynamic, goal_mode, length, width, wheelbase, start_state, goal_state,
control_bounds), `obstacles` (a list discriminated by `type`), `solver` (N, dt, use_slack,
slack_penalty, use_smooth, smooth_weight, mode casadi | l4casadi, initializer list, enforce_heading,
type ipopt | sqpmethod) and `model` (the learned-SDF architecture the reference would train).
"""
from __future__ import annotations

import math
from enum import Enum
from typing import List, Literal, Optional, Tuple, Union

import yaml
from pydantic import BaseModel, Field, RootModel

from .problem import Problem


class Dynamics(str, Enum):  # core/dynamics.py:7-13
    POINT_1ST = "point_1st"
    POINT_2ND = "point_2nd"
    UNICYCLE = "unicycle"
    UNICYCLE_2ND = "unicycle_2nd"
    ACKERMANN = "ackermann"
    ACKERMANN_2ND = "ackermann_2nd"


class Shape(str, Enum):  # core/geometry.py:17-20
    DOT = "dot"
    RECTANGLE = "rectangle"
    TRIANGLE = "triangle"


class GoalMode(str, Enum):  # core/geometry.py:12-14 (carried, unused by the NLP as in the reference)
    CENTER = "center"
    ANY_POINT = "any_point"


class Body(BaseModel):
    shape: Shape
    dynamic: Dynamics
    goal_mode: GoalMode = GoalMode.CENTER
    length: Optional[float] = None
    width: Optional[float] = None
    wheelbase: Optional[float] = None
    start_state: List[float]
    goal_state: List[float]
    control_bounds: List[Tuple[float, float]]


class Circle(BaseModel):
    type: Literal["circle"]
    center: Tuple[float, float]
    radius: float
    margin: float = 0.0


class Square(BaseModel):
    type: Literal["square"]
    center: Tuple[float, float]
    size: float
    margin: float = 0.0


class PolygonObs(BaseModel):
    type: Literal["polygon"]
    points: List[Tuple[float, float]]
    margin: float = 0.0


class EllipticRing(BaseModel):
    type: Literal["elliptical_ring"]
    center: Tuple[float, float]
    semi_axes: Tuple[float, float]
    width: float
    angle: float = math.pi
    margin: float = 0.0
    rotation: float = 0.0
    num_arc_points: int = 15


class DiscreteS(BaseModel):
    type: Literal["discr_s"]
    center: Tuple[float, float]
    semi_axes: Tuple[float, float]
    width: float
    angle: float = math.pi
    margin: float = 0.0
    rotation: float = 0.0
    num_arc_points: int = 30


class Trapezoid(BaseModel):
    type: Literal["trapezoid"]
    points: List[Tuple[float, float]]
    margin: float = 0.0


class Obstacles(RootModel[List[Union[Circle, Square, PolygonObs, EllipticRing, Trapezoid, DiscreteS]]]):
    pass


class DefaultInit(BaseModel):
    mode: Literal["default"] = "default"


class LinearInit(BaseModel):
    mode: Literal["linear"] = "linear"


class RRTInit(BaseModel):
    mode: Literal["rrt"] = "rrt"
    rrt_bounds: List[List[float]]
    step_size: float = Field(0.05, ge=1e-6)
    max_iter: int = Field(1000, ge=1)
    margin: float = Field(0.01, ge=0.0)


class Initializer(RootModel[List[Union[DefaultInit, LinearInit, RRTInit]]]):
    @property
    def choice(self):
        return self.root[0]


class Solver(BaseModel):
    N: int = Field(20, ge=1)
    dt: float = 0.1
    use_slack: bool = False
    slack_penalty: Optional[float] = Field(1000, ge=1)
    use_smooth: bool = False
    smooth_weight: float = Field(10.0, ge=0)
    mode: Literal["casadi", "l4casadi"]
    initializer: Initializer = Field(default_factory=lambda: Initializer(root=[LinearInit()]))
    enforce_heading: bool = True
    type: Literal["ipopt", "sqpmethod"]


class Model(BaseModel):
    type: Literal["mlp", "fourier", "siren"] = "mlp"
    hidden_dim: int = Field(64, ge=1)
    num_hidden_layers: int = Field(3, ge=1)
    activation_function: str = "ReLU"
    omega_0: float = 30.0
    n_samples: int = 200_000
    boundary_fraction: float = 0.3
    surface_loss_weight: float = Field(1.0, ge=0.0)
    eikonal_loss_weight: float = Field(1.0, ge=0.0)


class Config(BaseModel):
    body: Body
    obstacles: Obstacles
    solver: Solver
    model: Model

    @staticmethod
    def load(path) -> "Config":
        with open(path) as f:
            return Config(**yaml.safe_load(f))

    def obstacle_dicts(self):
        return [o.model_dump() for o in self.obstacles.root]

    def to_problem(self) -> Problem:
        """The NLP of RunBenchmark built from this config (run_benchmark.py:128-143)."""
        b, s = self.body, self.solver
        kw = dict(dynamics=b.dynamic.value, shape=b.shape.value, N=s.N, dt=s.dt, use_slack=s.use_slack,
                  slack_penalty=float(s.slack_penalty if s.slack_penalty is not None else 0.0),
                  use_smooth=s.use_smooth, smooth_weight=s.smooth_weight, enforce_heading=s.enforce_heading,
                  control_bounds=tuple(tuple(map(float, cb)) for cb in b.control_bounds),
                  sdf="mlp" if s.mode == "l4casadi" else "analytic")
        if b.shape != Shape.DOT:
            kw.update(length=float(b.length), width=float(b.width))
        if b.wheelbase is not None:
            kw["wheelbase"] = float(b.wheelbase)
        # the exact scene travels with the problem in both modes (the analytic SDF in casadi mode; the
        # learned SDF's training targets / sampling in l4casadi mode, where only the MLP enters the NLP)
        kw["obstacles"] = self.obstacle_dicts()
        return Problem(**kw)

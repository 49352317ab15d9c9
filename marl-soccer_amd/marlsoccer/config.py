"""config.json (soccer_simulation/config.json) -> ms_config.

Key semantics follow the reference exactly: keys read with [] there are required here,
keys read with .get(...) fall back to the same code defaults:
  physics.max_velocity/agent_mass/ball_mass/agent_friction/ball_friction  entities.py:11-17, 62-67 ([])
  physics.action_force_max      soccer_env.py:63  .get(..., 150000.0)
  physics.action_torque_max     soccer_env.py:64  .get(..., 100000.0)
  physics.max_angular_velocity  game.py:264       .get(..., action_torque_max / 100)
  rewards.ball_proximity_multiplier  game.py:330  .get(..., 0.0)
  rewards.move_ball_to_goal_multiplier, goal_scored_reward, goal_conceded_penalty,
  alive_penalty                 game.py:346, 365, 368, 372 ([])
  rewards.score_difference_multiplier  game.py:430  .get(..., 5.0)
  simulation.max_steps          game.py:27 ([])
"""
from __future__ import annotations

import copy
import json
import os

from . import _native as N

DEFAULT_CONFIG_PATH = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "config.json")


def load_config(path: str | None = None) -> dict:
    with open(path or DEFAULT_CONFIG_PATH) as f:
        return json.load(f)


def to_ms_config(config: dict, autoreset: bool) -> N.MsConfig:
    ph = config["physics"]
    rw = config["rewards"]
    c = N.MsConfig()
    c.max_velocity = float(ph["max_velocity"])
    c.agent_mass = float(ph["agent_mass"])
    c.ball_mass = float(ph["ball_mass"])
    c.agent_moment = 100.0  # entities.py:11
    c.ball_moment = 10.0  # entities.py:62
    c.agent_friction = float(ph["agent_friction"])
    c.ball_friction = float(ph["ball_friction"])
    c.agent_elasticity = 0.2  # entities.py:31
    c.agent_surface_friction = 0.8  # entities.py:32
    c.ball_elasticity = 0.95  # entities.py:80
    c.ball_surface_friction = 0.2  # entities.py:81
    c.action_force_max = float(ph.get("action_force_max", 150000.0))
    c.action_torque_max = float(ph.get("action_torque_max", 100000.0))
    c.max_angular_velocity = float(ph.get("max_angular_velocity", ph.get("action_torque_max", 100000.0) / 100.0))
    c.ball_proximity_multiplier = float(rw.get("ball_proximity_multiplier", 0.0))
    c.move_ball_to_goal_multiplier = float(rw["move_ball_to_goal_multiplier"])
    c.alive_penalty = float(rw["alive_penalty"])
    c.goal_scored_reward = float(rw["goal_scored_reward"])
    c.goal_conceded_penalty = float(rw["goal_conceded_penalty"])
    c.score_difference_multiplier = float(rw.get("score_difference_multiplier", 5.0))
    c.max_steps = int(config["simulation"]["max_steps"])
    c.autoreset = 1 if autoreset else 0
    return c


def resolve(config: dict | None) -> dict:
    return copy.deepcopy(config) if config is not None else load_config()

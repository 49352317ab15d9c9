"""Loading helpers for the committed golden fixtures (tests/golden/*.npz)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

CFG_MAP = {
    "physics.max_velocity": "max_velocity", "physics.agent_mass": "agent_mass",
    "physics.ball_mass": "ball_mass", "physics.agent_friction": "agent_friction",
    "physics.ball_friction": "ball_friction", "physics.action_torque_max": "action_torque_max",
    "rewards.ball_proximity_multiplier": "ball_proximity_multiplier",
    "rewards.move_ball_to_goal_multiplier": "move_ball_to_goal_multiplier",
    "rewards.alive_penalty": "alive_penalty", "rewards.goal_scored_reward": "goal_scored_reward",
    "rewards.goal_conceded_penalty": "goal_conceded_penalty",
    "rewards.score_difference_multiplier": "score_difference_multiplier",
    "simulation.max_steps": "max_steps",
}


def load(name):
    return np.load(os.path.join(GOLDEN, name), allow_pickle=False)


def traj_config_overrides(fx):
    """config.json key/values stored in a trajectory fixture -> ms_config field overrides."""
    out = {}
    for k, v in zip(fx["cfg_keys"], fx["cfg_vals"]):
        k = str(k)
        if k in CFG_MAP:
            out[CFG_MAP[k]] = int(v) if k == "simulation.max_steps" else float(v)
    if "action_torque_max" in out:
        out["max_angular_velocity"] = out["action_torque_max"] / 100.0
    return out


TRAJ_NAMES = ["default", "fullrandom", "fixed", "notrunc"]

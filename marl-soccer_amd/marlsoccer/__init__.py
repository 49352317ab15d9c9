"""marlsoccer — MI355X-native batched 2v2 soccer environment (host side).

GPU-resident batch API:         marlsoccer.SoccerBatch (frame-ring obs: FrameRingBatch)
Reference drop-ins (numpy/dict): soccer_env.SoccerEnv / soccerenv / make_env /
                                 get_observation_scalers, marl_vecenv.SyncMultiAgentVecEnv
                                 (modules at the root of marl-soccer_amd/, importable the
                                 same way as the reference's soccer_simulation/ modules)
"""
from .batch import FrameRingBatch, SoccerBatch, StepOutput, spawn_mode  # noqa: F401
from .config import load_config, to_ms_config  # noqa: F401
from . import _native  # noqa: F401

__all__ = ["SoccerBatch", "FrameRingBatch", "StepOutput", "spawn_mode", "load_config", "to_ms_config"]
# marlsoccer.rollout (Agent, RunningMeanStd, DeviceRollout): the device-resident policy loop

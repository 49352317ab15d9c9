"""Device-resident policy rollout for the soccer env.

The reference's caller (marl-soccer.ipynb, the `train` cell) runs its PPO rollout on the host:
every step it copies the observations to numpy, normalises them there, runs the policy, copies
the actions back and builds a numpy (N, 4, 3) action array with uniform(-1, 1) actions for the
two untrained red agents (notebook L289-336). Here the same loop stays on the GPU: obs ->
normaliser -> actor/critic MLP (hipBLASLt GEMMs through torch) -> action assembly -> ms_step,
with the rollout storage laid out exactly as the notebook's (num_steps, num_envs, 2, ...).

Formats are the reference's, so its artefacts load unchanged:
  * `Agent` has the notebook's / eval.py's module tree (critic.*, actor_mean.*, actor_logstd),
    so `Agent.load_state_dict(torch.load(path, weights_only=True))` reads a reference
    `*.ppo_model` checkpoint (eval.py:17-47, 58-60);
  * `RunningMeanStd.save_npz/load_npz` use the `mean`, `var` float64 (66,) arrays of
    `latest_normalizer_stats.npz` (notebook L455-458, eval.py:62-66).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn as nn
from torch.distributions.normal import Normal

from .policy import rollout_record

OBS_DIM, ACT_DIM = 66, 3
TRAINABLE = (0, 1)   # agent_0, agent_1 (blue) — notebook L243
RANDOM = (2, 3)      # red agents act uniformly at random — notebook L315-316


class RunningMeanStd:
    """Welford/Chan running moments, float64 on the device (notebook L190-222)."""

    def __init__(self, shape=(OBS_DIM,), device=None):
        self.device = torch.device("cpu") if device is None else torch.device(device)
        self.mean = torch.zeros(shape, dtype=torch.float64, device=self.device)
        self.var = torch.ones(shape, dtype=torch.float64, device=self.device)
        self.count = 0

    def update(self, x: torch.Tensor) -> None:
        """x: (B, *shape). np.mean / np.var(ddof=0) of the batch, then the notebook's merge."""
        x = x.to(self.device, torch.float64).reshape(-1, *self.mean.shape)
        batch_mean = x.mean(dim=0)
        batch_var = x.var(dim=0, unbiased=False)
        batch_count = x.shape[0]
        delta = batch_mean - self.mean
        tot_count = self.count + batch_count
        m_a = self.var * self.count
        m_b = batch_var * batch_count
        m2 = m_a + m_b + torch.square(delta) * self.count * batch_count / tot_count
        # in place: a captured rollout graph (DeviceRollout(graph=True)) reads these tensors
        self.mean.copy_(self.mean + delta * batch_count / tot_count)
        self.var.copy_(m2 / tot_count)
        self.count = tot_count

    @property
    def std(self) -> torch.Tensor:
        return torch.sqrt(self.var)

    def normalize(self, x: torch.Tensor) -> torch.Tensor:
        """clip((x - mean) / (std + 1e-8), -10, 10), in float64 then float32 (notebook L301:
        the rollout normalises the numpy float64 way before torch.tensor(..., dtype=float))."""
        y = (x.to(torch.float64) - self.mean) / (self.std + 1e-8)
        return torch.clamp(y, -10.0, 10.0).to(torch.float32)

    def save_npz(self, path: str) -> None:
        np.savez(path, mean=self.mean.cpu().numpy(), var=self.var.cpu().numpy())

    @classmethod
    def load_npz(cls, path: str, device=None) -> "RunningMeanStd":
        with np.load(path) as d:  # allow_pickle=False (numpy default)
            r = cls(tuple(d["mean"].shape), device)
            r.mean = torch.as_tensor(np.asarray(d["mean"], np.float64), device=r.device)
            r.var = torch.as_tensor(np.asarray(d["var"], np.float64), device=r.device)
        return r


def layer_init(layer: nn.Linear, std=np.sqrt(2), bias_const=0.0) -> nn.Linear:
    nn.init.orthogonal_(layer.weight, std)
    nn.init.constant_(layer.bias, bias_const)
    return layer


class Agent(nn.Module):
    """The reference's actor-critic (notebook `Agent`, eval.py:17-47): two tanh MLPs
    66-512-256-128-64-{1, 3} and a state-independent log-std."""

    def __init__(self, obs_dim: int = OBS_DIM, act_dim: int = ACT_DIM, rpo_alpha: float = 0.0):
        super().__init__()
        self.critic = nn.Sequential(
            layer_init(nn.Linear(obs_dim, 512)), nn.Tanh(),
            nn.Linear(512, 256), nn.Tanh(), nn.Linear(256, 128), nn.Tanh(),
            layer_init(nn.Linear(128, 64)), nn.Tanh(), layer_init(nn.Linear(64, 1), std=1.0),
        )
        self.actor_mean = nn.Sequential(
            layer_init(nn.Linear(obs_dim, 512)), nn.Tanh(),
            nn.Linear(512, 256), nn.Tanh(), nn.Linear(256, 128), nn.Tanh(),
            layer_init(nn.Linear(128, 64)), nn.Tanh(), layer_init(nn.Linear(64, act_dim), std=0.01),
        )
        self.actor_logstd = nn.Parameter(torch.zeros(1, act_dim))
        self.rpo_alpha = rpo_alpha

    def get_value(self, x: torch.Tensor) -> torch.Tensor:
        return self.critic(x)

    def get_action_and_value(self, x: torch.Tensor, action: torch.Tensor | None = None, generator=None):
        """notebook `get_action_and_value` (RPO: uniform(-alpha, alpha) jitter of the mean when
        re-evaluating a given action)."""
        action_mean = self.actor_mean(x)
        action_std = torch.exp(self.actor_logstd.expand_as(action_mean))
        if action is None:
            action = self._draw(action_mean, action_std, generator)
        else:
            z = (torch.rand(action_mean.shape, device=action_mean.device, generator=generator) * 2 - 1) * self.rpo_alpha
            action_mean = action_mean + z
        # no argument validation: it synchronises with the host (twice per call), which costs a
        # stall per rollout step and is not allowed inside a captured graph; values are unchanged
        probs = Normal(action_mean, action_std, validate_args=False)
        return action, probs.log_prob(action).sum(1), probs.entropy().sum(1), self.critic(x)

    @staticmethod
    def _draw(action_mean, action_std, generator):
        # torch.normal(mean, std, generator) computed as its kernels do (a standard normal draw,
        # times std, plus mean) without its host-side check that std >= 0, which synchronises
        # and cannot run inside a captured graph
        eps = torch.randn(action_mean.shape, device=action_mean.device, generator=generator)
        return eps * action_std + action_mean

    def sample(self, action_mean: torch.Tensor, generator=None):
        """get_action_and_value's sampled action and its log-prob, from a given actor mean."""
        action_std = torch.exp(self.actor_logstd.expand_as(action_mean))
        action = self._draw(action_mean, action_std, generator)
        return action, Normal(action_mean, action_std, validate_args=False).log_prob(action).sum(1)

    def get_deterministic_action(self, x: torch.Tensor) -> torch.Tensor:
        return self.actor_mean(x)


class DeviceRollout:
    """The notebook's rollout phase (L289-336) with every tensor on the env's device.

    collect() runs num_steps env steps and returns the PPO storage
    {obs, actions, logprobs, rewards, dones, values} shaped (num_steps, N, 2, ...) like the
    notebook's, plus next_obs / next_done for bootstrapping, the number of finished env
    episodes and the sum of their final (blue, red) scores.
    deterministic=True uses the actor mean (eval.py:79-81) instead of sampling.
    policy_dtype=torch.bfloat16 (opt-in; the notebook's policy is fp32, the default): the actor
    and critic GEMMs run under bf16 autocast (fp32 accumulation; normalisation, sampling,
    log-probs and storage stay fp32) — about half the forward's time; the action mean stays
    within 2e-4 and the value within 2e-2 of fp32 (the bound tests/test_policy.py asserts).
    graph=True: the first collect() runs eagerly (it also initialises the GEMM libraries); the
    second captures its num_steps steps as one HIP graph and replays it, and later calls replay
    that graph — one launch per rollout instead of ~40 kernel launches per step. The captured
    graph reads the agent's parameters and the normalizer's mean/var in place, so the PPO
    update must modify them in place (optimizer steps and RunningMeanStd.update do); a replay
    checks that those tensors are still the captured ones and captures again if not.
    policy="fused" (the default for fp32): the normalisation and both MLPs run as ONE gfx950
    kernel (ms_policy_forward: f32-input MFMA, activations in registers; marlsoccer.policy),
    within 1e-5 of the torch modules; "torch": the modules themselves (hipBLASLt GEMMs).
    Deviation of "fused": its tanh is the exp2/rcp form (~2e-7 absolute) and its log-prob uses
    logstd directly instead of log(exp(logstd)), so the stored logprobs and values differ from the
    torch Agent's by up to ~1e-5; a PPO update that recomputes log-probs with the torch modules
    (the notebook's) starts its first epoch with exp(new - old) within 1e-4 of 1, not exactly 1
    (tests/test_policy.py::test_fused_rollout_ppo_first_epoch_ratio_near_one). policy="torch"
    keeps the notebook's bit-for-bit first-epoch ratio of 1.
    """

    def __init__(self, batch, agent: Agent, normalizer: RunningMeanStd, num_steps: int, seed: int = 0,
                 deterministic: bool = False, update_normalizer: bool = True, graph: bool = False,
                 policy_dtype: torch.dtype = torch.float32, policy: str | None = None):
        self.batch, self.agent, self.normalizer = batch, agent, normalizer
        self.T, self.N = int(num_steps), batch.num_envs
        self.deterministic = deterministic
        self.update_normalizer = update_normalizer
        self.graph = graph
        if policy_dtype not in (torch.float32, torch.bfloat16):
            raise ValueError(f"policy_dtype must be torch.float32 or torch.bfloat16, got {policy_dtype}")
        self.policy_dtype = policy_dtype
        if policy is None:
            policy = "fused" if policy_dtype == torch.float32 else "torch"
        if policy not in ("fused", "torch") or (policy == "fused" and policy_dtype != torch.float32):
            raise ValueError(f"policy must be 'fused' (fp32) or 'torch', got {policy!r} with {policy_dtype}")
        self.policy = policy
        self._fused = None
        if policy == "fused":
            from .policy import FusedPolicy
            self._fused = FusedPolicy(agent)
            self._den = torch.ones((OBS_DIM,), dtype=torch.float64, device=batch.device)
        self._graph = None
        self._graph_inputs = None
        self._collects = 0
        dev = batch.device
        self.gen = torch.Generator(device=dev)
        self.gen.manual_seed(seed)
        T, N = self.T, self.N
        self.obs = torch.zeros((T, N, 2, OBS_DIM), dtype=torch.float32, device=dev)
        self.actions = torch.zeros((T, N, 2, ACT_DIM), dtype=torch.float32, device=dev)
        self.logprobs = torch.zeros((T, N, 2), dtype=torch.float32, device=dev)
        self.rewards = torch.zeros((T, N, 2), dtype=torch.float32, device=dev)
        self.dones = torch.zeros((T, N, 2), dtype=torch.float32, device=dev)
        self.values = torch.zeros((T, N, 2), dtype=torch.float32, device=dev)
        self.full_actions = torch.zeros((N, 4, ACT_DIM), dtype=torch.float32, device=dev)
        self.next_obs = batch.obs[:, list(TRAINABLE)].clone()
        self.next_done = torch.zeros((N, 2), dtype=torch.float32, device=dev)
        self.episodes = torch.zeros((), dtype=torch.int64, device=dev)  # finished env episodes
        self.score_sum = torch.zeros((2,), dtype=torch.int64, device=dev)

    @torch.no_grad()
    def step(self, t: int) -> None:
        b = self.batch
        if self._fused is None or t == 0:  # the fused step's record launch writes row t + 1
            self.dones[t] = self.next_done
        if self._fused is None:
            self.obs[t] = self.next_obs
        if self._fused is not None:
            # ONE kernel: normalisation, actor, critic, sampling and log-prob, straight from the
            # env's (N, 4, 66) obs rows of the blue agents into the storage and the env's actions
            # (the same generator draws as the torch path: eps, then the red agents' uniforms)
            eps = None if self.deterministic else torch.randn((2 * self.N, ACT_DIM), device=b.device, generator=self.gen)
            red = torch.rand((2 * self.N, ACT_DIM), generator=self.gen, device=b.device)
            self._fused.run(b.obs, 2 * self.N, 2, 264, 66, self.normalizer.mean, self._den, eps=eps,
                            action=self.actions[t], logprob=self.logprobs[t], value=self.values[t],
                            obs_copy=self.obs[t], env_actions=self.full_actions, red_uniform=red)
            b.step_into(self.full_actions, b.obs, b.rew, b.term, b.trunc, b.goal, b.score)
            # ONE launch for the step's rewards, dones and finished-episode counters
            rollout_record(b.rew, b.term, b.trunc, b.score, self.rewards[t], self.next_done,
                           self.dones[t + 1] if t + 1 < self.T else None, self.episodes, self.score_sum)
            return
        else:
            x = self.normalizer.normalize(self.next_obs.reshape(-1, OBS_DIM))
            # no autocast weight-cast cache: its casts would be allocated and reused across a graph
            # capture (the casts of ~0.4 M parameters per step are negligible)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.policy_dtype == torch.bfloat16,
                                cache_enabled=False):
                if self.deterministic:
                    action = self.agent.get_deterministic_action(x)
                    value = self.agent.get_value(x)
                    logprob = torch.zeros(x.shape[0], device=x.device)
                else:
                    action_mean = self.agent.actor_mean(x).float()
                    value = self.agent.get_value(x)
        if not self.deterministic:
            action, logprob = self.agent.sample(action_mean, generator=self.gen)
        self.values[t] = value.reshape(self.N, 2)
        self.actions[t] = action.reshape(self.N, 2, ACT_DIM)
        self.logprobs[t] = logprob.reshape(self.N, 2)
        fa = self.full_actions
        fa[:, :2] = self.actions[t]
        fa[:, 2:] = torch.rand((self.N, 2, ACT_DIM), generator=self.gen, device=fa.device) * 2.0 - 1.0
        b.step_into(fa, b.obs, b.rew, b.term, b.trunc, b.goal, b.score)
        self.rewards[t] = b.rew[:, :2]
        self.next_obs.copy_(b.obs[:, :2])
        done = (b.term[:, :2] | b.trunc[:, :2]).to(torch.float32)
        self.next_done.copy_(done)
        finished = b.trunc[:, 0].to(torch.bool)  # episodes end together for all four agents
        self.episodes += finished.sum()
        self.score_sum += (b.score * finished[:, None]).sum(dim=0)

    @torch.no_grad()
    def _run_steps(self) -> None:
        if self._fused is not None:  # the parameters and the normaliser as they are now
            self._fused.pack()
            torch.add(self.normalizer.std, 1e-8, out=self._den)
        for t in range(self.T):
            self.step(t)
        if self._fused is not None:  # the fused step reads the env's obs rows directly
            self.next_obs.copy_(self.batch.obs[:, :2])

    def _inputs_identity(self) -> tuple:
        """The tensors a captured rollout reads in place (their storage)."""
        return tuple(p.data_ptr() for p in self.agent.parameters()) + (self.normalizer.mean.data_ptr(),
                                                                          self.normalizer.var.data_ptr())

    def _capture(self) -> None:
        b, dev = self.batch, self.batch.device
        g = torch.cuda.CUDAGraph()
        g.register_generator_state(self.gen)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        old = b.stream
        b.set_stream(s)  # ms_step launches on the capture stream
        try:
            with torch.cuda.graph(g, stream=s):
                self._run_steps()
        finally:
            b.set_stream(old)
        torch.cuda.current_stream(dev).wait_stream(s)
        self._graph = g

    def collect(self) -> dict:
        if self.graph and self._collects > 0:
            if self._graph is not None and self._graph_inputs != self._inputs_identity():
                self._graph = None  # parameters or normaliser tensors were replaced: capture again
            if self._graph is None:
                self._capture()  # records only; the replay below runs it
                self._graph_inputs = self._inputs_identity()
            self._graph.replay()
        else:
            self._run_steps()
        self._collects += 1
        # the policy's actions are checked once per rollout (one synchronisation): a non-finite
        # action raises the reference's ValueError (soccer_env.py:116-117)
        self.batch.raise_if_nonfinite()
        if self.update_normalizer:  # notebook L347: after the rollout, from the raw observations
            self.normalizer.update(self.obs.reshape(-1, OBS_DIM))
        return {"obs": self.obs, "actions": self.actions, "logprobs": self.logprobs, "rewards": self.rewards,
                "dones": self.dones, "values": self.values, "next_obs": self.next_obs, "next_done": self.next_done,
                "episodes": self.episodes, "score_sum": self.score_sum}

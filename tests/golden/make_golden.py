"""Generate the golden fixtures in tests/golden/ from the REFERENCE's own Python code.

Run in the build container only (needs /root/reference, read-only):
    python tests/golden/make_golden.py

The reference (soccer_simulation/game/game.py, soccer_env.py, marl_vecenv.py, and the
velocity callbacks of game/entities.py) is imported unmodified. Its third-party imports
are absent here and are replaced by stand-ins defined in this file:
  - pygame, gymnasium, pettingzoo: import-level stubs (headless; spaces.Box; ParallelEnv)
  - pymunk: a shim. Body/Vec2d/Space bookkeeping restates pymunk's behaviour; Space.step
    runs the oracle's f64 Chipmunk restatement (oracle/liborc_f64.so) in two phases and,
    between them, calls each body's Python velocity_func exactly where cpSpaceStep does,
    so entities.py's damping/clamp code runs as the reference wrote it.
Physics numerics vs real Chipmunk stay "parity unpinned" (pymunk is unpinned and not
installed); everything the reference computes in Python — spawn RNG draws, observations,
reward shaping, goal/terminal logic, frame stacking, vec auto-reset — is pinned by these
fixtures.

Nothing here ships: only the .npz outputs are committed.
"""
from __future__ import annotations

import ctypes as C
import math
import os
import sys
import types
from typing import NamedTuple

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference/soccer_simulation"
sys.path.insert(0, os.path.join(REPO, "oracle"))
import oracle as orc  # noqa: E402

# ----------------------------------------------------------------------------------------
# import stubs
# ----------------------------------------------------------------------------------------
pygame = types.ModuleType("pygame")
pygame.init = lambda: None
pygame.quit = lambda: None
pygame.display = types.SimpleNamespace(set_mode=lambda *a, **k: None, set_caption=lambda *a: None,
                                       flip=lambda: None)
pygame.time = types.SimpleNamespace(Clock=lambda: None)
pygame.draw = types.SimpleNamespace(line=lambda *a, **k: None, circle=lambda *a, **k: None,
                                    rect=lambda *a, **k: None, polygon=lambda *a, **k: None)
sys.modules["pygame"] = pygame

gymnasium = types.ModuleType("gymnasium")
gspaces = types.ModuleType("gymnasium.spaces")


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), np.dtype(dtype)


gspaces.Box = Box
gymnasium.spaces = gspaces
sys.modules["gymnasium"] = gymnasium
sys.modules["gymnasium.spaces"] = gspaces

pettingzoo = types.ModuleType("pettingzoo")


class ParallelEnv:
    pass


pettingzoo.ParallelEnv = ParallelEnv
sys.modules["pettingzoo"] = pettingzoo

# ----------------------------------------------------------------------------------------
# pymunk shim
# ----------------------------------------------------------------------------------------
pymunk = types.ModuleType("pymunk")


class Vec2d(NamedTuple):
    x: float
    y: float

    def __add__(self, o):
        if isinstance(o, np.ndarray):
            return NotImplemented
        return Vec2d(self.x + o[0], self.y + o[1])

    def __sub__(self, o):
        if isinstance(o, np.ndarray):
            return NotImplemented
        return Vec2d(self.x - o[0], self.y - o[1])

    def __mul__(self, s):
        return Vec2d(self.x * s, self.y * s)

    __rmul__ = __mul__

    def __truediv__(self, s):
        return Vec2d(self.x / s, self.y / s)

    def __neg__(self):
        return Vec2d(-self.x, -self.y)

    @property
    def length(self):
        return math.sqrt(self.x * self.x + self.y * self.y)

    def normalized(self):
        ln = self.length
        return self / ln if ln != 0 else Vec2d(0.0, 0.0)

    def get_distance(self, o):
        return math.sqrt((self.x - o[0]) ** 2 + (self.y - o[1]) ** 2)


def _v(t):
    return Vec2d(float(t[0]), float(t[1]))


class Body:
    DYNAMIC, KINEMATIC, STATIC = 0, 1, 2

    def __init__(self, mass=0, moment=0, body_type=0):
        self.mass, self.moment, self.body_type = mass, moment, body_type
        self._p = Vec2d(0.0, 0.0)
        self._v = Vec2d(0.0, 0.0)
        self._a = 0.0
        self._w = 0.0
        self._f = Vec2d(0.0, 0.0)
        self._t = 0.0
        self._vb = (0.0, 0.0)
        self._wb = 0.0
        self._vfunc = Body.update_velocity
        self.shapes = []

    position = property(lambda s: s._p, lambda s, v: setattr(s, "_p", _v(v)))
    velocity = property(lambda s: s._v, lambda s, v: setattr(s, "_v", _v(v)))
    force = property(lambda s: s._f, lambda s, v: setattr(s, "_f", _v(v)))
    angle = property(lambda s: s._a, lambda s, v: setattr(s, "_a", float(v)))
    angular_velocity = property(lambda s: s._w, lambda s, v: setattr(s, "_w", float(v)))
    torque = property(lambda s: s._t, lambda s, v: setattr(s, "_t", float(v)))
    velocity_func = property(lambda s: s._vfunc, lambda s, f: setattr(s, "_vfunc", f))

    @staticmethod
    def update_velocity(body, gravity, damping, dt):
        """cpBodyUpdateVelocity: v = v*damping + (g + f*m_inv)*dt; w = w*damping + t*i_inv*dt."""
        m_inv = 1.0 / body.mass
        i_inv = 1.0 / body.moment
        vx = body._v.x * damping + (gravity[0] + body._f.x * m_inv) * dt
        vy = body._v.y * damping + (gravity[1] + body._f.y * m_inv) * dt
        body._v = Vec2d(vx, vy)
        body._w = body._w * damping + body._t * i_inv * dt
        body._f = Vec2d(0.0, 0.0)
        body._t = 0.0

    def apply_force_at_local_point(self, force, point=(0, 0)):
        """cpBodyApplyForceAtLocalPoint at the body's centre: f += R(angle) force."""
        assert tuple(point) == (0, 0)
        c, s = math.cos(self._a), math.sin(self._a)
        fx = c * force[0] + (-s) * force[1]
        fy = s * force[0] + c * force[1]
        self._f = Vec2d(self._f.x + fx, self._f.y + fy)

    def local_to_world(self, v):
        c, s = math.cos(self._a), math.sin(self._a)
        return Vec2d(c * v[0] - s * v[1] + self._p.x, s * v[0] + c * v[1] + self._p.y)


class ShapeFilter(NamedTuple):
    group: int = 0
    categories: int = 0xFFFFFFFF
    mask: int = 0xFFFFFFFF


class Shape:
    def __init__(self, body):
        self.body = body
        self.elasticity = 0.0
        self.friction = 0.0
        self.filter = ShapeFilter()
        self.collision_type = 0


class Poly(Shape):
    @staticmethod
    def create_box(body, size, radius=0):
        p = Poly(body)
        p.size, p.radius = tuple(size), radius
        return p


class Circle(Shape):
    def __init__(self, body, radius, offset=(0, 0)):
        super().__init__(body)
        self.radius = radius


class Segment(Shape):
    def __init__(self, body, a, b, radius):
        super().__init__(body)
        self.a, self.b, self.radius = tuple(map(float, a)), tuple(map(float, b)), float(radius)


_ORC = orc.load("f64")
_CFG = orc.default_config()
_PARAMS = (C.c_char * _ORC.orc_sizeof_params())()
_ORC.orc_params_init(C.byref(_CFG), _PARAMS)


class _OrcBody(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("px", "py", "vx", "vy", "a", "w", "vbx", "vby", "wb", "fx", "fy", "t")]


EXPECTED_STATICS = [((10.0, 10.0), (790.0, 10.0), 2.0), ((10.0, 590.0), (790.0, 590.0), 2.0),
                    ((10.0, 10.0), (10.0, 225.0), 2.0), ((10.0, 375.0), (10.0, 590.0), 2.0),
                    ((790.0, 10.0), (790.0, 225.0), 2.0), ((790.0, 375.0), (790.0, 590.0), 2.0),
                    ((10.0, 225.0), (10.0, 375.0), 1.0), ((790.0, 225.0), (790.0, 375.0), 1.0)]


class Space:
    def __init__(self):
        self.gravity = (0, 0)
        self.static_body = Body(body_type=Body.STATIC)
        self.bodies = []
        self.shapes = []
        self.statics = []
        self._mem = (C.c_char * _ORC.orc_sizeof_space())()
        self._bod = (_OrcBody * 5).from_buffer(self._mem)

    def add(self, *objs):
        for o in objs:
            if isinstance(o, Body):
                self.bodies.append(o)
            elif isinstance(o, Segment):
                self.statics.append(o)
                i = len(self.statics) - 1
                a, b, r = EXPECTED_STATICS[i]
                assert (o.a, o.b, o.radius) == (a, b, r), (o.a, o.b, o.radius)
            else:
                self.shapes.append(o)

    def remove(self, *objs):
        for o in objs:
            if isinstance(o, Body):
                self.bodies.remove(o)
            else:
                self.shapes.remove(o)
        _ORC.orc_space_clear_arbiters(self._mem)  # cpSpaceFilterArbiters for removed bodies

    def _ordered(self):
        agents = [s.body for s in self.shapes if isinstance(s, Poly)]
        balls = [s.body for s in self.shapes if isinstance(s, Circle)]
        assert len(agents) == 4 and len(balls) == 1
        return agents + balls

    def _push(self, bodies):
        for ob, b in zip(self._bod, bodies):
            ob.px, ob.py, ob.vx, ob.vy = b._p.x, b._p.y, b._v.x, b._v.y
            ob.a, ob.w, ob.vbx, ob.vby, ob.wb = b._a, b._w, b._vb[0], b._vb[1], b._wb
            ob.fx, ob.fy, ob.t = b._f.x, b._f.y, b._t

    def _pull(self, bodies):
        for ob, b in zip(self._bod, bodies):
            b._p, b._v = Vec2d(ob.px, ob.py), Vec2d(ob.vx, ob.vy)
            b._w, b._vb, b._wb = ob.w, (ob.vbx, ob.vby), ob.wb
            if b is not bodies[4]:
                b._a = ob.a
            b._f, b._t = Vec2d(ob.fx, ob.fy), ob.t

    def step(self, dt):
        assert dt == 1 / 60.0
        bodies = self._ordered()
        self._push(bodies)
        _ORC.orc_space_phase1(self._mem, _PARAMS)
        self._pull(bodies)
        for b in self.bodies:  # cpSpaceStep: body->velocity_func(body, gravity, damping, dt)
            b.velocity_func(b, self.gravity, 1.0, dt)
        self._push(bodies)
        _ORC.orc_space_phase2(self._mem, _PARAMS)
        self._pull(bodies)


pymunk.Vec2d, pymunk.Body, pymunk.Space = Vec2d, Body, Space
pymunk.Poly, pymunk.Circle, pymunk.Segment, pymunk.ShapeFilter = Poly, Circle, Segment, ShapeFilter
sys.modules["pymunk"] = pymunk

# ----------------------------------------------------------------------------------------
# reference imports
# ----------------------------------------------------------------------------------------
sys.path.insert(0, REF)
from game.game import Game  # noqa: E402
import marl_vecenv  # noqa: E402
import soccer_env  # noqa: E402

with open(os.path.join(REF, "config.json")) as f:
    import json
    CONFIG = json.load(f)


def rng_state(g):
    st = g.bit_generator.state
    s, i = int(st["state"]["state"]), int(st["state"]["inc"])
    m = (1 << 64) - 1
    return np.array([s >> 64, s & m, i >> 64, i & m, st["has_uint32"], st["uinteger"]], dtype=np.uint64)


def game_positions(game):
    return np.array([tuple(a.body.position) for a in game.agents] + [tuple(game.ball.body.position)])


# ----------------------------------------------------------------------------------------
# 1. spawn / RNG fixtures (game.py:76-249)
# ----------------------------------------------------------------------------------------
def make_spawn():
    seeds = [0, 1, 7, 19, 20, 42, 12345, 2 ** 32 + 5, 2 ** 40 + 3]
    modes = {0: {}, 1: {"use_full_random_positions": True}, 2: {"use_fixed_positions": True}}
    n_soft = 12
    out_seed, out_mode, pos, ang, rng, pcg0 = [], [], [], [], [], []
    for seed in seeds:
        for mode, opt in modes.items():
            g = Game(CONFIG, headless=True)
            g.reset(seed=seed, **opt)
            p = [game_positions(g)]
            a = [[ag.body.angle for ag in g.agents]]
            r = [rng_state(g._rng)]
            for _ in range(n_soft):
                g._reset_positions()
                p.append(game_positions(g))
                a.append([ag.body.angle for ag in g.agents])
                r.append(rng_state(g._rng))
            out_seed.append(seed)
            out_mode.append(mode)
            pos.append(p)
            ang.append(a)
            rng.append(r)
            pcg0.append(rng_state(np.random.default_rng(seed))[:4])
    np.savez_compressed(os.path.join(HERE, "spawn.npz"), seed=np.array(out_seed, np.uint64),
                        mode=np.array(out_mode, np.int32), pos=np.array(pos), angle=np.array(ang),
                        rng=np.array(rng, dtype=np.uint64), pcg0=np.array(pcg0, dtype=np.uint64))
    print("spawn.npz", np.array(pos).shape)


# ----------------------------------------------------------------------------------------
# 2. observation fixtures (game.py:258-322 + soccer_env.py:131 fp32 cast)
# ----------------------------------------------------------------------------------------
def set_state(game, pos, vel, ang, w):
    for i, ag in enumerate(game.agents):
        ag.body.position = tuple(map(float, pos[i]))
        ag.body.velocity = tuple(map(float, vel[i]))
        ag.body.angle = float(ang[i])
        ag.body.angular_velocity = float(w[i])
    game.ball.body.position = tuple(map(float, pos[4]))
    game.ball.body.velocity = tuple(map(float, vel[4]))


def safe_angles(r, n):
    a = r.uniform(-20, 20, n).astype(np.float32)
    wrap = np.abs(np.remainder(a.astype(np.float64) + np.pi, 2 * np.pi) - np.pi)
    a[np.abs(wrap - np.pi) < 1e-3] = 0.5  # keep away from the atan2 branch cut
    return a


def make_obs():
    r = np.random.default_rng(1234)
    n = 400
    pos = r.uniform([5, 5], [795, 595], (n, 5, 2)).astype(np.float32)
    vel = r.uniform(-260, 260, (n, 5, 2)).astype(np.float32)
    ang = np.stack([safe_angles(r, 4) for _ in range(n)]).astype(np.float64)
    ang[:8] = 0.0
    ang[8:16, 2:] = math.pi  # spawn facing of the red team (f64 pi; fp32 state holds fl32(pi))
    w = r.uniform(-25, 25, (n, 4)).astype(np.float32)
    # special cases: coincident bodies (unit vector (0,0), mag 0), bodies on the goal points
    pos[16, 1] = pos[16, 0]
    pos[17, 4] = pos[17, 2]
    pos[18, 0] = (10, 300)
    pos[19, 3] = (790, 300)
    pos[20, 0] = pos[20, 4] + np.float32(1e-6)
    g = Game(CONFIG, headless=True)
    g.reset(seed=0)
    frames = np.zeros((n, 4, 22), np.float32)
    for k in range(n):
        set_state(g, pos[k], vel[k], ang[k], w[k])
        obs = g._get_observations()
        frames[k] = np.asarray(obs, dtype=np.float32)
    np.savez_compressed(os.path.join(HERE, "obs.npz"), pos=pos, vel=vel, angle=ang, w=w, frames=frames)
    print("obs.npz", frames.shape)


# ----------------------------------------------------------------------------------------
# 3. reward fixtures (game.py:251-256, 324-375, 424-433)
# ----------------------------------------------------------------------------------------
def make_rewards():
    r = np.random.default_rng(99)
    n = 600
    prev = r.uniform([15, 15], [785, 585], (n, 5, 2)).astype(np.float32)
    step = r.uniform(-4, 4, (n, 5, 2)).astype(np.float32)
    cur = (prev + step).astype(np.float32)
    goal = r.integers(0, 3, n).astype(np.int8)
    goal[:200] = 0
    prev[300:310, 4] = (790, 300)  # ball on the red goal point before / after
    cur[310:320, 4] = (790, 300)
    cur[320:330, 0] = cur[320:330, 4]  # agent on the ball
    out = np.zeros((n, 2))
    configs = {"default": dict(CONFIG), "conceded": json.loads(json.dumps(CONFIG))}
    configs["conceded"]["rewards"]["goal_conceded_penalty"] = 1.5
    configs["conceded"]["rewards"]["ball_proximity_multiplier"] = 0.0
    res = {}
    for name, cfg in configs.items():
        g = Game(cfg, headless=True)
        g.reset(seed=0)
        zero = np.zeros((5, 2))
        for k in range(n):
            set_state(g, prev[k], zero, np.zeros(4), np.zeros(4))
            g._update_reward_state()
            set_state(g, cur[k], zero, np.zeros(4), np.zeros(4))
            info = {"scored": False}
            if goal[k] == 1:
                info = {"scored": True, "scoring_team_color": (0, 0, 255)}
            elif goal[k] == 2:
                info = {"scored": True, "scoring_team_color": (255, 0, 0)}
            out[k] = g._calculate_rewards(info)
        res[name] = out.copy()
    np.savez_compressed(os.path.join(HERE, "rewards.npz"), prev=prev, cur=cur, goal=goal,
                        rew_default=res["default"], rew_conceded=res["conceded"])
    print("rewards.npz", n)


# ----------------------------------------------------------------------------------------
# 4. trajectory fixtures: SyncMultiAgentVecEnv over SoccerEnv over Game (shim physics)
# ----------------------------------------------------------------------------------------
def controller(game, rng, chase):
    """Deterministic goal-seeking actions for agents in `chase`, random for the others."""
    acts = rng.uniform(-1, 1, (4, 3)).astype(np.float32)
    ball = np.array(tuple(game.ball.body.position))
    for i in chase:
        body = game.agents[i].body
        p = np.array(tuple(body.position))
        goal = np.array([790.0, 300.0]) if i < 2 else np.array([10.0, 300.0])
        to_goal = goal - ball
        to_goal /= np.linalg.norm(to_goal) + 1e-9
        behind = ball - 24.0 * to_goal
        d = behind - p
        if np.linalg.norm(d) < 6.0 or np.dot(ball - p, to_goal) > 0 and np.linalg.norm(ball - p) < 30:
            d = ball - p + 20 * to_goal
        d = d / (np.linalg.norm(d) + 1e-9)
        c, s = math.cos(body.angle), math.sin(body.angle)
        local = np.array([c * d[0] + s * d[1], -s * d[0] + c * d[1]])
        acts[i, :2] = np.clip(local * 1.2, -1, 1)
        acts[i, 2] = np.clip(-0.5 * body.angular_velocity, -1, 1)
    return acts


def make_traj(name, n_envs, n_steps, seed, options, cfg_over):
    chasers = [(0,), (2,), (1,), (3,), (0, 2)]
    cfg = json.loads(json.dumps(CONFIG))
    for sect, kv in cfg_over.items():
        cfg[sect].update(kv)
    envs = marl_vecenv.SyncMultiAgentVecEnv([lambda: soccer_env.soccerenv(config=cfg) for _ in range(n_envs)])
    obs0 = envs.reset(options=options, seed=seed)
    r = np.random.default_rng(seed + 10 ** 6)
    A = np.zeros((n_steps, n_envs, 4, 3), np.float32)
    O = np.zeros((n_steps, n_envs, 4, 66), np.float32)
    R = np.zeros((n_steps, n_envs, 4))
    TE = np.zeros((n_steps, n_envs, 4), bool)
    TR = np.zeros((n_steps, n_envs, 4), bool)
    G = np.zeros((n_steps, n_envs), np.int8)
    S = np.zeros((n_steps, n_envs, 2), np.int32)
    P = np.zeros((n_steps, n_envs, 5, 2))
    for t in range(n_steps):
        for e, env in enumerate(envs.envs):
            A[t, e] = controller(env._game, r, chasers[e % len(chasers)])
        o, rw, te, tr, infos = envs.step(A[t])
        O[t], R[t], TE[t], TR[t] = o, rw, te, tr
        for e, env in enumerate(envs.envs):
            inf = infos[e]["agent_0"]
            S[t, e] = inf["score"]["blue"], inf["score"]["red"]
            gb = inf.get("goal_scored_by")
            G[t, e] = 0 if gb is None else (1 if gb == "blue" else 2)
            assert all(infos[e][a] == inf for a in envs.possible_agents)
            P[t, e] = game_positions(env._game)
    pcg = np.stack([rng_state(np.random.default_rng(seed + i))[:4] for i in range(n_envs)])
    mode = 2 if options and options.get("use_fixed_positions") else (1 if options and options.get("use_full_random_positions") else 0)
    flat = {f"{s}.{k}": v for s, kv in cfg.items() for k, v in kv.items()}
    np.savez_compressed(os.path.join(HERE, f"traj_{name}.npz"), obs0=obs0, actions=A, obs=O, rew=R,
                        term=TE, trunc=TR, goal=G, score=S, pos=P, pcg=pcg, mode=np.int32(mode),
                        cfg_keys=np.array(list(flat.keys())), cfg_vals=np.array([float(v) for v in flat.values()]))
    print(f"traj_{name}.npz envs={n_envs} steps={n_steps} goals={int((G != 0).sum())} "
          f"dones={int(TR[..., 0].sum())} obs0={obs0.shape}")


if __name__ == "__main__":
    make_spawn()
    make_obs()
    make_rewards()
    make_traj("default", 2, 1010, 19, None, {})
    make_traj("fullrandom", 6, 500, 7, {"use_full_random_positions": True},
              {"simulation": {"max_steps": 200}, "rewards": {"score_difference_multiplier": 5.0,
                                                              "goal_conceded_penalty": 1.0}})
    make_traj("fixed", 2, 400, 3, {"use_fixed_positions": True},
              {"simulation": {"max_steps": 150}, "rewards": {"score_difference_multiplier": 2.0}})
    make_traj("notrunc", 4, 900, 11, None, {"simulation": {"max_steps": 0}})

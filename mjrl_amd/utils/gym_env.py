"""EnvSpec — the policy / baseline constructor input (mjrl/utils/gym_env.py:4-9).

GymEnv itself (the MuJoCo env wrapper) stays with the reference: sampling runs on
host CPUs through the reference's samplers (out of scope)."""


class EnvSpec(object):
    def __init__(self, obs_dim, act_dim, horizon, num_agents):
        self.observation_dim = obs_dim
        self.action_dim = act_dim
        self.horizon = horizon
        self.num_agents = num_agents

"""mjrl_amd — MI355X (gfx950) NPG / TRPO / DAPG update path with mjrl's API.

    from mjrl_amd.policies.gaussian_mlp import MLP
    from mjrl_amd.algos.npg_cg import NPG          # TRPO, DAPG, BatchREINFORCE alike
    agent = NPG(env, MLP(env.spec, (64, 64)), baseline, normalized_step_size=0.1)
    agent.train_step(N=50, gae_lambda=0.97)         # drop-in for mjrl's train_agent loop

The update runs in hand-written HIP kernels through the C ABI of
include/mjrl_amd.h (library: mjrl_amd/lib/libmjrl_amd.so, built by
`python -m mjrl_amd.build`).  There is no CPU fallback.
"""
__version__ = "0.1.0"

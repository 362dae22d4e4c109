"""omniisaacgymenvs_amd — MI355X-native replacement for the PhysX GPU pipeline + task layer
behind OmniIsaacGymEnvs' VecEnvBase / RLTask (Humanoid, Ant, Cartpole).

Layout: csrc/ (HIP kernels + C ABI of libmi_sim.so, declared in include/mi_sim.h),
native.py (ctypes binding; fails loudly without the HIP library), robots/ (MJCF-subset model
compiler, ArticulationView, GridCloner), tasks/ + envs/ (the reference's Python surface),
utils/ (Hydra-compatible config composition, task registry, rl_games adapter).
"""
__version__ = "0.1.0"

"""MI355X-native DPPO fine-tuning hot path (diffusion-policy sampler + PPO update) as gfx950 HIP
kernels behind a C ABI (include/dppo.h), with the reference's Python class surface
(agent.finetune.TrainPPODiffusionAgent, model.diffusion.PPODiffusion, DiffusionMLP, CriticObs)
mirrored under this package so Hydra-style configs stay drop-in."""
__version__ = "0.1.0"

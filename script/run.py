"""Entry point with the reference's CLI (script/run.py:33-88):
    python script/run.py --config-name=ft_ppo_diffusion_mlp --config-dir=cfg/gym/finetune/hopper-v2 [key=value ...]
Hydra/OmegaConf are replaced by diffusionpolicyoptimization_amd.util.config (same YAML, same
_target_ strings, same resolvers); the dataset/checkpoint downloads (:44-74) are skipped (no
network): a missing base policy falls back to seeded synthetic weights with a warning."""
import argparse
import logging
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

from diffusionpolicyoptimization_amd.util.config import get_class, load_config  # noqa: E402


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--config-name", required=True)
    ap.add_argument("--config-dir", "--config-path", dest="config_dir", default=os.path.join(os.getcwd(), "cfg"))
    args, overrides = ap.parse_known_args(argv)
    logging.basicConfig(level=logging.INFO, format="[%(asctime)s][%(name)s][%(levelname)s] - %(message)s")
    cfg = load_config(args.config_dir, args.config_name, overrides)
    agent = get_class(cfg._target_)(cfg)
    return agent.run()


if __name__ == "__main__":
    main()

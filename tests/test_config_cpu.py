"""codenerf.config.load_config: the reference's YAML keys (config/srn-cars-code.yml layout) as attributes,
the CLI keys of train.py:182-201 first, overrides merged last."""
import textwrap

from codenerf.config import Cfg, load_config


def test_load_config_layout(tmp_path):
    p = tmp_path / "c.yml"
    p.write_text(textwrap.dedent("""
        experiment:
            id: x
            randomseed: 55
            iterations: 500000
        dataset:
            basedir: /data/srn_cars
            train_batch_size: 4
        optimizer:
            type: AdamW
            lr: 1.0E-4
        nerf:
            point_sampler:
                num_coarse: 32
                spacing_mode: "lindepth"
                perturb: True
    """))
    cfg = load_config(str(p), gpus=2, is_distributed=True, nerf={"point_sampler": {"num_coarse": 64}})
    assert cfg.gpus == 2 and cfg.is_distributed and cfg.load_checkpoint == ""
    assert cfg.experiment.randomseed == 55 and cfg.dataset.train_batch_size == 4
    assert cfg.optimizer.lr == 1e-4 and cfg.optimizer.type == "AdamW"
    assert cfg.nerf.point_sampler.num_coarse == 64 and cfg.nerf.point_sampler.spacing_mode == "lindepth"
    assert cfg.nerf.point_sampler.perturb is True
    assert "angle_lr" not in cfg.optimizer and not hasattr(cfg.optimizer, "angle_lr")
    c2 = cfg | {"load_checkpoint": "a.ckpt"}
    assert isinstance(c2, Cfg) and c2.load_checkpoint == "a.ckpt" and cfg.load_checkpoint == ""
    assert c2.nerf.point_sampler.num_coarse == 64

import os

import yaml

from .models import Config, DataConfig, DiffusionConfig, FolderConfig, ModelConfig, TrainingConfig

DEFAULT_CONFIG_PATH = os.path.join(os.path.dirname(__file__), 'config.yaml')


def load_config(config_path: str = DEFAULT_CONFIG_PATH) -> Config:
    """YAML -> validated ``Config`` (reference ``sample_ddpm.py:17-20``)."""
    with open(config_path, 'r') as fh:
        return Config(**yaml.safe_load(fh))


def model_config(im_size: int = 128, **overrides) -> ModelConfig:
    """The default ``config.yaml`` model section with ``im_size`` (and any field) overridden."""
    base = load_config().model.model_dump()
    base['im_size'] = im_size
    base.update(overrides)
    return ModelConfig(**base)


__all__ = [
    'Config', 'DataConfig', 'DiffusionConfig', 'FolderConfig', 'ModelConfig', 'TrainingConfig',
    'load_config', 'model_config', 'DEFAULT_CONFIG_PATH'
]

"""Pydantic configuration schema, field-for-field compatible with the reference.

Mirrors ``diffusion_model/config/models.py:5-66`` of xXCoffeeColaXc/WeatherConverter so the same
``config.yaml`` validates unchanged.  Build-only knobs (backend, noise mode, world size) are NOT
added here: they live as keyword arguments of the sampling API so the YAML schema stays the
reference's.
"""
from typing import List, Optional

from pydantic import BaseModel


class DataConfig(BaseModel):  # reference config/models.py:5-13
    root_dir: str
    acdc_dir: str
    acdc_labels: str
    acdc_images: str
    bdd_dir: str
    dawn_dir: str
    weather: List[str]
    image_size: List[int]


class DiffusionConfig(BaseModel):  # reference config/models.py:16-19
    num_timesteps: int
    beta_start: float
    beta_end: float


class ModelConfig(BaseModel):  # reference config/models.py:22-34
    name: str
    im_channels: int
    im_size: int
    down_channels: List[int]
    mid_channels: List[int]
    down_sample: List[bool]
    time_emb_dim: int
    num_down_layers: int
    num_mid_layers: int
    num_up_layers: int
    num_heads: int
    attn_resolutions: List[int]


class FolderConfig(BaseModel):  # reference config/models.py:37-42
    output: str
    weights: str
    logs: str
    checkpoints: str
    samples: str


class TrainingConfig(BaseModel):  # reference config/models.py:45-58
    device: str = 'cuda'
    random_seed: int
    epochs: int
    batch_size: int
    num_workers: int
    lr: float
    log_interval: int
    save_interval: int
    sample_interval: int
    resume_training: bool
    resume_checkpoint: Optional[str] = None
    sample_size: int
    num_grid_rows: int


class Config(BaseModel):  # reference config/models.py:61-66
    training: TrainingConfig
    diffusion: DiffusionConfig
    data: DataConfig
    model: ModelConfig
    folders: FolderConfig

from .linear_noise_scheduler import LinearNoiseScheduler

__all__ = ['LinearNoiseScheduler']

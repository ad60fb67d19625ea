from .sgg import apply_gsg, apply_lcg

__all__ = ['apply_gsg', 'apply_lcg']

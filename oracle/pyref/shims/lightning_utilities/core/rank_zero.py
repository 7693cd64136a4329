import warnings


def rank_zero_warn(msg, *args, **kwargs):
    warnings.warn(str(msg))

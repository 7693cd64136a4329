# Off-path (torch_cluster is used only by Distance / GN / T models, out of scope).
def radius_graph(*args, **kwargs):
    raise NotImplementedError("torch_cluster is not available; not on the ET/TensorNet hot path")

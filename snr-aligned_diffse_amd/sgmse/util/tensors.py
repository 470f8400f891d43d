def batch_broadcast(a, x):
    """Broadcast a per-batch tensor `a` [B] against `x` [B, ...] (reference util/tensors.py)."""
    if len(a.shape) != 1:
        a = a.squeeze()
        if len(a.shape) != 1:
            raise ValueError(f"Don't know how to batch-broadcast tensor `a` with more than one effective dimension (shape {a.shape})")
    if a.shape[0] != x.shape[0] and a.shape[0] != 1:
        raise ValueError(f"Don't know how to batch-broadcast shape {a.shape} over {x.shape} as the batch dimension is not matching")
    return a.view([-1] + [1] * (len(x.shape) - 1))

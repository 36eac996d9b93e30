"""Checkpoint I/O for the clip models (reference: train_visual.py:629-636, train_audio.py:87,
train_au_face.py:748-756, test_au_face.py:107-141).

The models keep the reference's 288-key NCHW ``state_dict`` (the kernels' NHWC / packed
weight layouts are derived on the device and never saved), so the reference's files load
here and files saved here load into the reference.  Loading never unpickles code:
``torch.load(..., weights_only=True)`` only.

``unwrap_state_dict`` / ``load_state_dict_flexible`` restate test_au_face.py:107-141 (EMA,
Lightning and DataParallel containers) with one deliberate difference: the reference strips
the first seven characters of EVERY key once any container is unwrapped
(``new_state[kk[7:]] = ...``, test_au_face.py:123), which truncates keys without a
``module.`` prefix; here only ``module.``-prefixed keys are stripped (the two agree whenever
every key carries the prefix, the case the reference handles).

``save_training_state`` / ``load_training_state`` add what the reference never saves
(optimizer, GradScaler, scheduler, epoch) so a run can resume.
"""
import torch

CONTAINER_KEYS = ["state_dict", "model", "ema_state_dict", "model_ema", "ema", "net", "module"]


def unwrap_state_dict(raw):
    state = raw
    for k in CONTAINER_KEYS:   # test_au_face.py:110-113
        if isinstance(state, dict) and k in state and isinstance(state[k], dict):
            state = state[k]
    if isinstance(state, dict):
        state = {k: v for k, v in state.items() if k != "n_averaged"}   # :116-117
        state = {(k[7:] if k.startswith("module.") else k): v for k, v in state.items()}   # :120-124 (see above)
    return state


def load_state_dict_flexible(model, path_or_state, verbose=True):
    """test_au_face.py:128-141: strict load, falling back to strict=False (reporting what is
    missing / unexpected).  Returns the (missing, unexpected) key lists."""
    raw = path_or_state if isinstance(path_or_state, dict) else torch.load(path_or_state, map_location="cpu",
                                                                           weights_only=True)
    state = unwrap_state_dict(raw)
    try:
        model.load_state_dict(state, strict=True)
        return [], []
    except RuntimeError as e:
        if verbose:
            print(f"[Load] strict=True failed -> {e.__class__.__name__}: {str(e).splitlines()[0]}")
        missing, unexpected = model.load_state_dict(state, strict=False)
        if verbose:
            print(f"[Load] strict=False | missing={len(missing)} unexpected={len(unexpected)}")
        return list(missing), list(unexpected)


def save_training_state(path, model, optimizer=None, scaler=None, scheduler=None, epoch=None, **extra):
    """{"model": state_dict, ...} in the reference's container layout (train_visual.py:633-636)
    plus the state needed to resume."""
    ck = {"model": model.state_dict()}
    if optimizer is not None:
        ck["optimizer"] = optimizer.state_dict()
    if scaler is not None:
        ck["scaler"] = scaler.state_dict()
    if scheduler is not None:
        ck["scheduler"] = scheduler.state_dict()
    if epoch is not None:
        ck["epoch"] = int(epoch)
    for k, v in extra.items():
        ck[k] = v.state_dict() if hasattr(v, "state_dict") else v
    torch.save(ck, path)


def load_training_state(path, model, optimizer=None, scaler=None, scheduler=None, map_location="cpu"):
    ck = torch.load(path, map_location=map_location, weights_only=True)
    model.load_state_dict(ck["model"])
    if optimizer is not None and "optimizer" in ck:
        optimizer.load_state_dict(ck["optimizer"])
    if scaler is not None and "scaler" in ck:
        scaler.load_state_dict(ck["scaler"])
    if scheduler is not None and "scheduler" in ck:
        scheduler.load_state_dict(ck["scheduler"])
    return ck

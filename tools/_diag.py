"""DFWFM_DIAG helpers for the diagnostics tools (the library reads one "key=value,..." variable)."""
import os


def diag_get(key, default=None):
    """One option of the library's DFWFM_DIAG="key=value,..." test / diagnostics list."""
    for kv in os.environ.get("DFWFM_DIAG", "").split(","):
        k, _, v = kv.partition("=")
        if k == key:
            return v
    return default


def diag_set(key, value, overwrite=True):
    if not overwrite and diag_get(key) is not None:
        return
    kept = [kv for kv in os.environ.get("DFWFM_DIAG", "").split(",") if kv and kv.partition("=")[0] != key]
    os.environ["DFWFM_DIAG"] = ",".join(kept + [f"{key}={value}"])

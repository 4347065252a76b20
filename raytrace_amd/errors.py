"""Error types mirroring the C-ABI status codes (include/rt.h RT_E_*)."""


class RtError(RuntimeError):
    code = -1


class RtInvalid(RtError, ValueError):
    """RT_E_INVALID: malformed scene / camera (the reference would `error` or produce NaNs)."""
    code = -2


class RtUnsupported(RtError):
    """RT_E_UNSUPPORTED: a closure the device cannot evaluate (custom material / texture /
    background, non-Euclidean transform).  The reference's own CPU path is the fallback."""
    code = -3


class RtDeviceError(RtError):
    """RT_E_HIP: a HIP runtime failure, or the HIP library / GPU is missing."""
    code = -4

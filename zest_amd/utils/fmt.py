"""Human-readable sizes and rates (decimal GB, as reported by bench.py)."""


def human_bytes(n: float) -> str:
    for unit in ("B", "KB", "MB", "GB", "TB"):
        if abs(n) < 1000 or unit == "TB":
            return f"{n:.1f} {unit}" if unit != "B" else f"{int(n)} B"
        n /= 1000.0
    return f"{n:.1f} TB"


def human_rate(nbytes: float, seconds: float) -> str:
    return human_bytes(nbytes / seconds if seconds > 0 else 0.0) + "/s"

"""Learning-rate schedule (reference ballbot_rl/training/schedules.py:4-19).

progress_remaining runs from 1 (start) to 0 (end): 1e-4 above 0.7, 5e-5 strictly
between 0.5 and 0.7, else 1e-5 -- including exactly 0.7, which the reference's
strict comparisons send to the last branch.
"""


def lr_schedule(progress_remaining: float) -> float:
    if progress_remaining > 0.7:
        return 1e-4
    if 0.5 < progress_remaining < 0.7:
        return 5e-5
    return 1e-5

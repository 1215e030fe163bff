"""Time-axis resampling helper of the 2-D dataset path (reference data/transforms.py:135-147)."""


def get_t_downsample(tmin, tmax, nt_in, nt_out=None, ratio_nt=None):
    """(first, last) time of a uniform nt_in-point time axis on [tmin, tmax] kept every `ratio_nt`-th point
    (ratio_nt = nt_in / nt_out when only nt_out is given; it must be integral).  Point i of the axis is
    tmin + (i / (nt_in - 1)) * (tmax - tmin), evaluated in that order so the floats equal the
    reference's."""
    if ratio_nt is None:
        if nt_out is None:
            raise ValueError("Either nt_out or ratio_nt must be specified")
        ratio_nt = nt_in / nt_out
    if not isinstance(ratio_nt, int):
        if not float(ratio_nt).is_integer():
            raise AssertionError(f"time downsampling ratio {ratio_nt} is not an integer")
        ratio_nt = int(ratio_nt)
    span = tmax - tmin
    last = ((nt_in - 1) // ratio_nt) * ratio_nt  # index of the last kept point

    def t_at(i):
        return tmin + (i / (nt_in - 1) * span)

    return t_at(0), t_at(last)

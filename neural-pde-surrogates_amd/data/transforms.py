"""The one transform helper the 2-D dataset path uses (reference data/transforms.py:135-147)."""


def get_t_downsample(tmin, tmax, nt_in, nt_out=None, ratio_nt=None):
    tdelta = tmax - tmin
    range_old = [tmin + (x / (nt_in - 1) * tdelta) for x in range(0, nt_in)]
    if nt_out is None and ratio_nt is None:
        raise ValueError("Either nt_out or ratio_nt must be specified")
    elif ratio_nt is None:
        ratio_nt = nt_in / nt_out
    if not isinstance(ratio_nt, int):
        assert ratio_nt.is_integer()
        ratio_nt = int(ratio_nt)
    range_new = range_old[::ratio_nt]
    return range_new[0], range_new[-1]

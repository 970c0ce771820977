"""Window-size clamping (vst:72-85) shared by the modules and the kernel engine."""


def get_window_size(x_size, window_size, shift_size=None):
    """Clamp the window to the input on every dim where x <= window, and zero
    the shift there (so at D = 7 = Wd the D-shift becomes 0)."""
    use_window_size = list(window_size)
    use_shift_size = list(shift_size) if shift_size is not None else None
    for i in range(len(x_size)):
        if x_size[i] <= window_size[i]:
            use_window_size[i] = x_size[i]
            if use_shift_size is not None:
                use_shift_size[i] = 0
    if use_shift_size is None:
        return tuple(use_window_size)
    return tuple(use_window_size), tuple(use_shift_size)

"""Shim of the one more_itertools function the reference's extraction imports
(not installed here): locate(iterable, pred) yields the indices where pred holds.
Container-only (listed in .gpurunignore), like the filterpy shim."""


def locate(iterable, pred=bool, window_size=None):
    if window_size is not None:
        raise NotImplementedError("window_size")
    return (i for i, item in enumerate(iterable) if pred(item))

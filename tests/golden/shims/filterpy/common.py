"""filterpy.common stand-in: the reference imports the module but uses nothing from it."""


class Saver(object):
    def __init__(self, *a, **k):
        pass

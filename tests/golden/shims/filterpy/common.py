"""filterpy.common stand-in: the reference creates Saver objects and calls save()
(extract_track_candidates.py:210,223,288,311) but never reads what they record."""


class Saver(object):
    def __init__(self, *a, **k):
        pass

    def save(self):
        pass

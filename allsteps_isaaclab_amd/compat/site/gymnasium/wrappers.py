"""Shim of ``gymnasium.wrappers``: video recording needs a renderer, which the MI355X build has not."""


class RecordVideo:
    def __init__(self, *args, **kwargs):
        raise RuntimeError("--video: there is no renderer in the MI355X build (DESIGN.md §8)")

"""Robot base -- mirrors models/robot.py:8-43 (state/input containers, dt,
``transition``).  The model arithmetic runs in libvcmpc.so kernels."""
from __future__ import annotations

from abc import ABC, abstractmethod

from ..utils.fancy_vector import FancyVector


class Robot(ABC):
    def __init__(self, config):
        self.dt = config["dt"]
        self.config = config
        self.state: FancyVector = self.__class__.create_state()
        self.input: FancyVector = self.__class__.create_action()
        self._init_model()

    @abstractmethod
    def _init_model(self):
        pass

    @property
    @abstractmethod
    def transition(self):
        pass

    @classmethod
    @abstractmethod
    def create_state(cls, *args, **kwargs) -> FancyVector:
        pass

    @classmethod
    @abstractmethod
    def create_action(cls, *args, **kwargs) -> FancyVector:
        pass

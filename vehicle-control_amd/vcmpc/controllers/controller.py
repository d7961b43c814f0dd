"""Controller base -- mirrors controllers/controller.py:6-19 (``command`` contract).
``step`` is the north star's ``Controller.step(state) -> u`` alias."""
from abc import ABC, abstractmethod


class Controller(ABC):
    def __init__(self, kp=None, kd=None):
        self.kp = kp
        self.kd = kd

    @abstractmethod
    def command(self, *args, **kwargs):
        pass

    def step(self, state):
        return self.command(state)

"""Name -> class registry (API of the reference's sgmse/util/registry.py:5-34)."""
import warnings
from typing import Callable


class Registry:
    def __init__(self, managed_thing: str):
        self.managed_thing = managed_thing
        self._registry = {}

    def register(self, name: str) -> Callable:
        def inner(cls):
            if name in self._registry:
                warnings.warn(f"{self.managed_thing} with name '{name}' doubly registered, old class will be replaced.")
            self._registry[name] = cls
            return cls
        return inner

    def get_by_name(self, name: str):
        try:
            return self._registry[name]
        except KeyError:
            raise ValueError(f"{self.managed_thing} with name '{name}' unknown.") from None

    def get_all_names(self):
        return list(self._registry)

"""Cross-language handles (reference: python/ray/cross_language.py): ``java_function``,
``java_actor_class``, ``cpp_function``, ``cpp_actor_class`` describe remote code in another
language's worker. ray_amd runs Python workers only, so the handles can be built and
passed around, and calling ``.remote()`` raises ``CrossLanguageError``."""

from __future__ import annotations

from ray_amd.exceptions import CrossLanguageError


class _CrossLanguageHandle:
    def __init__(self, language: str, kind: str, *names: str):
        self.language, self.kind, self.names = language, kind, names

    def options(self, **kw):
        return self

    def remote(self, *args, **kwargs):
        raise CrossLanguageError(
            f"{self.language} {self.kind} {'.'.join(self.names)}: ray_amd has no "
            f"{self.language} workers (Python only)")

    def __repr__(self):
        return f"<{self.language} {self.kind} {'.'.join(self.names)}>"


def java_function(class_name: str, function_name: str):
    return _CrossLanguageHandle("Java", "function", class_name, function_name)


def java_actor_class(class_name: str):
    return _CrossLanguageHandle("Java", "actor class", class_name)


def cpp_function(function_name: str):
    return _CrossLanguageHandle("C++", "function", function_name)


def cpp_actor_class(create_function_name: str, class_name: str):
    return _CrossLanguageHandle("C++", "actor class", class_name, create_function_name)

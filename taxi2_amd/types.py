"""Core types mirrored from the reference (API contract only; no compute here).

* :class:`Type` / :class:`TypeMeta` restate ``itaxotools.common.types`` 0.3.4 as used by
  ``src/itaxotools/taxi2/types.py:5``: every direct subclass of a Type becomes an attribute of
  its parent (``DistanceMetric.Uncorrected``), ``for child in Parent`` iterates the direct
  subclasses (``distances.py:307``), ``Child in Parent`` tests membership, instances compare
  equal by type and ``obj.type`` is the class (``versus_all.py:601``).  Pinned by
  ``tests/test_types.py:8-37`` (restated in tests/test_host_api.py).
* :class:`Container` restates ``types.py:10-39``: a re-iterable source; a callable source is
  re-invoked on every ``__iter__`` and ``len()`` iterates the whole source.
"""

from __future__ import annotations

from typing import Callable, Generic, Iterable, Iterator, TypeVar

Item = TypeVar("Item")


class TypeMeta(type):
    _children: dict = {}

    def __new__(mcs, name, bases, namespace, **kwargs):
        cls = super().__new__(mcs, name, bases, namespace, **kwargs)
        TypeMeta._children[cls] = []
        for base in bases:
            if isinstance(base, TypeMeta):
                TypeMeta._children[base].append(cls)
                setattr(base, name, cls)
        return cls

    def __iter__(cls) -> Iterator[type]:
        return iter(list(TypeMeta._children.get(cls, ())))

    def __contains__(cls, item) -> bool:
        return any(item is child for child in TypeMeta._children.get(cls, ()))


class Type(metaclass=TypeMeta):
    """Registry base: subclasses are reachable as attributes of their parents."""

    def __eq__(self, other) -> bool:
        return type(self) is type(other)

    def __hash__(self) -> int:
        return hash(type(self))

    def __repr__(self) -> str:
        return f"<{type(self).__name__}>"

    @property
    def type(self) -> type:
        return type(self)


class Container(Generic[Item]):
    """Re-iterable lazy source (``types.py:10-39``)."""

    def __init__(self, source: Iterable[Item] | Callable[..., Iterator[Item]], *args, **kwargs):
        if callable(source):
            self._call = source
            self._iterable = None
            self._args, self._kwargs = args, kwargs
        else:
            if args or kwargs:
                raise TypeError("Cannot pass arguments to iterable source")
            self._call = None
            self._iterable = source
            self._args, self._kwargs = (), {}

    def __iter__(self) -> Iterator[Item]:
        if self._call is not None:
            return iter(self._call(*self._args, **self._kwargs))
        return iter(self._iterable)

    def __len__(self) -> int:
        return sum(1 for _ in self)


class AttrDict(dict):
    """``itaxotools.common.utility.AttrDict``: a dict whose keys are attributes."""

    def __getattr__(self, key):
        try:
            return self[key]
        except KeyError as e:
            raise AttributeError(key) from e

    def __setattr__(self, key, value):
        self[key] = value

    def __delattr__(self, key):
        del self[key]

"""The part of deppy's pkg/entitysource the resolution façade needs.

Mirrors pkg/entitysource/entity.go (Entity), cache_querier.go (CacheQuerier)
and entity_source.go:47-110 (Group).  The entity store itself is out of scope
(SURVEY.md §2); this is the lookup surface DeppySolver uses
(pkg/solver/solver.go:53-62).
"""
from __future__ import annotations

from typing import Callable, Dict, Iterable, List, Optional


class EntityID(str):
    pass


class EntityPropertyNotFoundError(Exception):
    def __init__(self, key: str):
        super().__init__("Property '(%s)' Not Found" % key)  # entity.go:10-12


class Entity:
    """entity.go:14-33"""

    def __init__(self, id: str, properties: Optional[Dict[str, str]] = None):
        self._id = EntityID(id)
        self._properties = dict(properties or {})

    def ID(self) -> EntityID:
        return self._id

    def GetProperty(self, key: str):
        if key not in self._properties:
            return "", EntityPropertyNotFoundError(key)
        return self._properties[key], None


class CacheQuerier:
    """cache_querier.go:7-53: an in-memory map of entities."""

    def __init__(self, entities: Dict[str, Entity]):
        self.entities = {EntityID(k): v for k, v in entities.items()}

    def Get(self, ctx, id) -> Optional[Entity]:
        return self.entities.get(EntityID(id))

    def Filter(self, ctx, predicate: Callable[[Entity], bool]):
        return [e for e in self.entities.values() if predicate(e)], None

    def GroupBy(self, ctx, fn: Callable[[Entity], Iterable[str]]):
        out: Dict[str, List[Entity]] = {}
        for e in self.entities.values():
            for key in fn(e):
                out.setdefault(key, []).append(e)
        return out, None

    def Iterate(self, ctx, fn: Callable[[Entity], Optional[Exception]]):
        for e in self.entities.values():
            err = fn(e)
            if err is not None:
                return err
        return None

    def GetContent(self, ctx, id):
        return None, None


class Group:
    """entity_source.go:47-110: sources queried in order, first hit wins."""

    def __init__(self, *sources):
        self.entitySources = list(sources)

    def Get(self, ctx, id) -> Optional[Entity]:
        for s in self.entitySources:
            e = s.Get(ctx, id)
            if e is not None:
                return e
        return None

    def Filter(self, ctx, predicate):
        out: List[Entity] = []
        for s in self.entitySources:
            rs, err = s.Filter(ctx, predicate)
            if err is not None:
                return None, err
            out.extend(rs)
        return out, None

    def GroupBy(self, ctx, fn):
        out: Dict[str, List[Entity]] = {}
        for s in self.entitySources:
            rs, err = s.GroupBy(ctx, fn)
            if err is not None:
                return None, err
            for k, v in rs.items():
                out.setdefault(k, []).extend(v)
        return out, None

    def Iterate(self, ctx, fn):
        for s in self.entitySources:
            err = s.Iterate(ctx, fn)
            if err is not None:
                return err
        return None


def NewGroup(*sources) -> Group:
    return Group(*sources)


def NewEntity(id: str, properties: Optional[Dict[str, str]] = None) -> Entity:
    return Entity(id, properties)


def NewCacheQuerier(entities: Dict[str, Entity]) -> CacheQuerier:
    return CacheQuerier(entities)

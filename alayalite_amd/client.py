"""Client: registry + persistence of indices (mirrors alayalite/client.py,
python/src/alayalite/client.py:28-294).  Collections (the pandas document layer above Index,
client.py:115-133 / collection.py) are outside this engine's scope."""

from __future__ import annotations

import json
import os
import shutil

from .index import Index
from .schema import IndexParams, is_collection_url, is_index_url

__all__ = ["Client"]

_NO_COLLECTIONS = "collections are not part of the MI355X engine (only the Index API is)"


class Client:
    """Manages named indices and, when constructed with a url, their on-disk copies."""

    def __init__(self, url=None):
        self.__index_map = {}
        self.__url = None
        if url is None:
            return
        self.__url = os.path.abspath(url)
        os.makedirs(self.__url, exist_ok=True)
        for name in sorted(os.listdir(self.__url)):
            full = os.path.join(self.__url, name)
            if not os.path.isdir(full):
                continue
            if is_index_url(full):
                self.__index_map[name] = Index.load(self.__url, name)
            elif is_collection_url(full):
                print(f"Collection {name} skipped: {_NO_COLLECTIONS}")
            else:
                print(f"Unknown url: {full} is found")

    def list_collections(self):
        return []

    def list_indices(self):
        return list(self.__index_map.keys())

    def get_collection(self, name: str = "default"):  # noqa: ARG002 - API parity
        return None

    def get_index(self, name: str = "default") -> Index:
        index = self.__index_map.get(name)
        if index is None:
            print(f"Index {name} does not exist")
        return index

    def create_collection(self, name: str = "default", **kwargs):
        raise RuntimeError(_NO_COLLECTIONS)

    def get_or_create_collection(self, name: str, **kwargs):
        raise RuntimeError(_NO_COLLECTIONS)

    def create_index(self, name: str = "default", **kwargs) -> Index:
        if name in self.__index_map:
            raise RuntimeError(f"A collection or index with name '{name}' already exists")
        index = Index(name, IndexParams.from_kwargs(**kwargs))
        self.__index_map[name] = index
        return index

    def get_or_create_index(self, name: str, **kwargs) -> Index:
        index = self.__index_map.get(name)
        return index if index is not None else self.create_index(name, **kwargs)

    def delete_collection(self, collection_name: str, delete_on_disk: bool = False):
        raise RuntimeError(f"Collection '{collection_name}' does not exist")

    def delete_index(self, index_name: str, delete_on_disk: bool = False):
        if index_name not in self.__index_map:
            raise RuntimeError(f"Index '{index_name}' does not exist")
        del self.__index_map[index_name]
        if delete_on_disk:
            if self.__url is None:
                raise RuntimeError("Client is not initialized with a url for disk operations")
            path = os.path.join(self.__url, index_name)
            if os.path.exists(path):
                shutil.rmtree(path)

    def reset(self, delete_on_disk: bool = False):
        if delete_on_disk and self.__url is None:
            raise RuntimeError("Client is not initialized with a url for disk operations")
        self.__index_map = {}

    def save_index(self, index_name: str):
        if self.__url is None:
            raise RuntimeError("Client is not initialized with a url")
        if index_name not in self.__index_map:
            raise RuntimeError(f"Index '{index_name}' does not exist")
        index_url = os.path.join(self.__url, index_name)
        schema_map = self.__index_map[index_name].save(index_url)
        with open(os.path.join(index_url, "schema.json"), "w", encoding="utf-8") as f:
            json.dump(schema_map, f, indent=4)

    def save_collection(self, collection_name: str):
        raise RuntimeError(_NO_COLLECTIONS)

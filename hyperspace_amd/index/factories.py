"""Dependency-injection seams (reference ``index/factories.scala:22-53``).

Tests replace these with fakes, exactly like the reference's Mockito-based action tests.
"""
from __future__ import annotations

from ..utils import file_utils as FU
from .data_manager import IndexDataManagerImpl
from .log_manager import IndexLogManagerImpl


class IndexLogManagerFactory:
    def create(self, index_path: str):
        raise NotImplementedError


class IndexLogManagerFactoryImpl(IndexLogManagerFactory):
    def create(self, index_path: str):
        return IndexLogManagerImpl(index_path)


class IndexDataManagerFactory:
    def create(self, index_path: str):
        raise NotImplementedError


class IndexDataManagerFactoryImpl(IndexDataManagerFactory):
    def create(self, index_path: str):
        return IndexDataManagerImpl(index_path)


class FileSystemFactory:
    def create(self, path: str):
        raise NotImplementedError


class FileSystemFactoryImpl(FileSystemFactory):
    def create(self, path: str):
        return FU.get_fs(path)

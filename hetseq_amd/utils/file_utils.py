"""Pretrained-artifact cache (reference: file_utils.py:78-226), offline-safe.

``cached_path`` resolves a local path, or a URL whose ETag-hashed copy is
already in the cache directory (``$PYTORCH_PRETRAINED_BERT_CACHE`` or
``~/.pytorch_pretrained_bert``, the reference's layout: file
``sha256(url)[.sha256(etag)]`` plus a ``.json`` sidecar).  Downloading is
attempted only for http(s) when ``requests`` is importable and the host is
reachable; S3 needs boto3, which is imported lazily (the reference imports
it at module load, Q30).
"""
from __future__ import annotations

import fnmatch
import hashlib
import json
import os
import shutil
import tempfile
from urllib.parse import urlparse

PYTORCH_PRETRAINED_BERT_CACHE = os.getenv(
    "PYTORCH_PRETRAINED_BERT_CACHE", os.path.join(os.path.expanduser("~"), ".pytorch_pretrained_bert"))


def url_to_filename(url, etag=None):
    filename = hashlib.sha256(url.encode("utf-8")).hexdigest()
    if etag:
        filename += "." + hashlib.sha256(etag.encode("utf-8")).hexdigest()
    return filename


def filename_to_url(filename, cache_dir=None):
    cache_dir = cache_dir or PYTORCH_PRETRAINED_BERT_CACHE
    meta_path = os.path.join(cache_dir, filename + ".json")
    if not os.path.exists(os.path.join(cache_dir, filename)) or not os.path.exists(meta_path):
        raise EnvironmentError("file {} not found".format(filename))
    with open(meta_path, encoding="utf-8") as f:
        metadata = json.load(f)
    return metadata["url"], metadata["etag"]


def _cached_copy(url, cache_dir):
    base = url_to_filename(url)
    if not os.path.isdir(cache_dir):
        return None
    hits = [f for f in fnmatch.filter(os.listdir(cache_dir), base + "*") if not f.endswith(".json")]
    return os.path.join(cache_dir, sorted(hits)[-1]) if hits else None


def cached_path(url_or_filename, cache_dir=None):
    cache_dir = str(cache_dir or PYTORCH_PRETRAINED_BERT_CACHE)
    url_or_filename = str(url_or_filename)
    parsed = urlparse(url_or_filename)
    if parsed.scheme in ("http", "https", "s3"):
        hit = _cached_copy(url_or_filename, cache_dir)
        if hit:
            return hit
        return get_from_cache(url_or_filename, cache_dir)
    if os.path.exists(url_or_filename):
        return url_or_filename
    if parsed.scheme == "":
        raise EnvironmentError("file {} not found".format(url_or_filename))
    raise ValueError("unable to parse {} as a URL or as a local path".format(url_or_filename))


def get_from_cache(url, cache_dir=None):
    cache_dir = cache_dir or PYTORCH_PRETRAINED_BERT_CACHE
    os.makedirs(cache_dir, exist_ok=True)
    if url.startswith("s3://"):
        try:
            import boto3  # noqa: F401  (lazy: optional dependency)
        except ImportError as e:
            raise EnvironmentError("s3:// URLs need boto3, which is not installed") from e
        raise EnvironmentError("offline: cannot fetch {}".format(url))
    import requests

    try:
        resp = requests.head(url, allow_redirects=True, timeout=5)
    except Exception as e:
        raise EnvironmentError("offline and no cached copy of {}".format(url)) from e
    etag = resp.headers.get("ETag")
    path = os.path.join(cache_dir, url_to_filename(url, etag))
    if not os.path.exists(path):
        with tempfile.NamedTemporaryFile() as tmp:
            r = requests.get(url, stream=True, timeout=30)
            for chunk in r.iter_content(chunk_size=1 << 20):
                tmp.write(chunk)
            tmp.flush()
            tmp.seek(0)
            with open(path, "wb") as out:
                shutil.copyfileobj(tmp, out)
        with open(path + ".json", "w", encoding="utf-8") as meta:
            json.dump({"url": url, "etag": etag}, meta)
    return path

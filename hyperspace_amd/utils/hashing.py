"""MD5 helper used by every signature provider.

Reference: ``util/HashingUtils.scala:24-35`` (commons-codec ``DigestUtils.md5Hex`` of the UTF-8
string).  Host-side on purpose: signatures fold O(#files) short strings.
"""
import hashlib


def md5_hex(value) -> str:
    return hashlib.md5(str(value).encode("utf-8")).hexdigest()

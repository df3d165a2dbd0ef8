"""audiotools.id3 — the ID3v2 prefix skip FLAC reading needs.

Only what sits on the decode path: a FLAC file may carry ID3v2 comments
in front of its "fLaC" marker (the reference's test/flac-id3.flac,
flac-id3-2.flac), which FlacAudio steps over before handing the stream to
the decoder (reference audiotools/flac.py:2433-2435, 1680-1684).
Tag editing is out of scope.
"""


def decode_syncsafe32(i):
    """a 32-bit sync-safe integer -> its 28-bit value; ValueError if any
    byte's top bit is set or the value is out of range
    (reference audiotools/id3.py:81-102)"""
    if i >= (1 << 32):
        raise ValueError("value of %s is too large" % i)
    if i < 0:
        raise ValueError("value cannot be negative")
    value = 0
    for x in range(4):
        if i & 0x80:
            raise ValueError("invalid sync-safe bit")
        value |= (i & 0x7F) << (x * 7)
        i >>= 8
    return value


def skip_id3v2_comment(file):
    """seek past every ID3v2 comment at the file's position; returns the
    bytes skipped, 0 (position restored) when there is none
    (reference audiotools/id3.py:264-310).  As in the reference, only the
    header's size field is read (no footer, no check of the tag body), and
    nested comments are skipped one after another."""
    start = file.tell()
    try:
        if file.read(3) != b"ID3":
            file.seek(start)
            return 0
        major = file.read(1)
        if len(major) < 1 or major[0] not in (2, 3, 4):
            file.seek(start)
            return 0
        file.read(1)   # minor version
        file.read(1)   # flags
        raw = file.read(4)
        try:
            if len(raw) < 4:
                raise ValueError("truncated size")
            # "32u" big-endian, then the sync-safe decode (least significant
            # byte first, as the reference's loop reads it)
            tag_size = decode_syncsafe32(int.from_bytes(raw, "big"))
        except ValueError:
            file.seek(start)
            return 0
        file.read(tag_size)
        return 10 + tag_size + skip_id3v2_comment(file)
    except IOError:
        file.seek(start)
        return 0

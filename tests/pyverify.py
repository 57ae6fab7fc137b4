"""Independent frame verifier (pure Python, RFC 791/768/793/792/1071).

Shares no code with the oracle or the kernels: parses a built frame field by
field and recomputes every checksum from the bytes, so a wrong composition in
both the oracle and the GPU path would still be caught here."""
import struct


def ones_sum(data: bytes) -> int:
    if len(data) & 1:
        data = data + b"\x00"
    s = sum(struct.unpack("!%dH" % (len(data) // 2), data))
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return s


def inet_csum(data: bytes) -> int:
    return (~ones_sum(data)) & 0xFFFF


def parse(frame: bytes) -> dict:
    d = {}
    d["dmac"], d["smac"], d["ethertype"] = frame[0:6], frame[6:12], struct.unpack("!H", frame[12:14])[0]
    ip = frame[14:34]
    (vihl, tos, tot, ident, frag, ttl, proto, csum) = struct.unpack("!BBHHHBBH", ip[:12])
    d.update(vihl=vihl, tos=tos, tot_len=tot, id=ident, frag=frag, ttl=ttl, proto=proto, ip_csum=csum,
             saddr=ip[12:16], daddr=ip[16:20])
    l4 = frame[34:]
    d["l4"] = l4
    if proto == 17:
        sp, dp, ln, ck = struct.unpack("!HHHH", l4[:8])
        d.update(sport=sp, dport=dp, udp_len=ln, l4_csum=ck, payload=l4[8:])
    elif proto == 6:
        sp, dp, sq, ak, off, flags, win, ck, urg = struct.unpack("!HHIIBBHHH", l4[:20])
        d.update(sport=sp, dport=dp, seq=sq, ack=ak, doff=off >> 4, flags=flags, window=win, l4_csum=ck, urg=urg,
                 payload=l4[20:])
    else:
        ty, co, ck = struct.unpack("!BBH", l4[:4])
        d.update(icmp_type=ty, icmp_code=co, l4_csum=ck, icmp_rest=l4[4:8], payload=l4[8:])
    return d


def ip_csum_ok(frame: bytes) -> bool:
    return ones_sum(frame[14:34]) == 0xFFFF


def l4_csum_value(frame: bytes) -> int:
    """The checksum a correct sender writes (RFC 768/793/792), check field treated as 0."""
    d = parse(frame)
    proto = d["proto"]
    l4 = bytearray(frame[34:])
    if proto == 17:
        l4[6:8] = b"\0\0"
    elif proto == 6:
        l4[16:18] = b"\0\0"
    else:
        l4[2:4] = b"\0\0"
        return inet_csum(bytes(l4))
    pseudo = d["saddr"] + d["daddr"] + struct.pack("!BBH", 0, proto, len(l4))
    return inet_csum(pseudo + bytes(l4))


def ip_csum_value(frame: bytes) -> int:
    h = bytearray(frame[14:34])
    h[10:12] = b"\0\0"
    return inet_csum(bytes(h))

"""Second, independent restatement of the per-iteration build in pure Python
(src/sequence.c:433-602) for small cases.  Written from
the spec, not from the C oracle, so the two cross-check each other."""
import socket
import struct

MASK32 = 0xFFFFFFFF
A, Cc = 1103515245, 12345


def rand_r(s):
    s = (s * A + Cc) & MASK32
    r = (s >> 16) & 0x7FF
    s = (s * A + Cc) & MASK32
    r = (r << 10) ^ ((s >> 16) & 0x3FF)
    s = (s * A + Cc) & MASK32
    r = (r << 10) ^ ((s >> 16) & 0x3FF)
    return r, s


def splitmix(x):
    z = (x + 0x9E3779B97F4A7C15) & (2**64 - 1)
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & (2**64 - 1)
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & (2**64 - 1)
    return z ^ (z >> 31)


def seed(base, seq, k):
    return splitmix(base ^ (((seq << 48) + k) & (2**64 - 1))) & MASK32


def rand_num(lo, hi, s):
    return rand_r(s)[0] % (hi - lo + 1) + lo


def csum(data):
    if len(data) & 1:
        data += b"\0"
    t = sum(struct.unpack("!%dH" % (len(data) // 2), data))
    while t >> 16:
        t = (t & 0xFFFF) + (t >> 16)
    return (~t) & 0xFFFF


def csum_single(hdr):
    t = sum(struct.unpack("!10H", hdr))
    return (~((t & 0xFFFF) + (t >> 16))) & 0xFFFF


def inet_aton(s):
    try:
        return struct.unpack("!I", socket.inet_aton(s))[0]
    except OSError:
        return None


def parse_range(r):
    if r is None:
        return None
    toks = [t for t in r.split("/") if t]
    if r.startswith("/") or len(toks) < 2:
        return None
    ip = inet_aton(toks[0])
    if ip is None:
        return None
    digits = ""
    for ch in toks[1].lstrip():
        if ch.isdigit() or (not digits and ch in "+-"):
            digits += ch
        else:
            break
    try:
        cidr = int(digits)
    except ValueError:
        cidr = 0
    if cidr < 0 or cidr > 32:
        return None
    hm = MASK32 if cidr == 0 else ((1 << (32 - cidr)) - 1)
    return ip & ~hm & MASK32, hm


def mac(s):
    return bytes(6) if not s else bytes(int(x, 16) for x in s.split(":"))


def exact_bytes(p):
    text = p["exact"]
    if p.get("isfile"):
        try:
            with open(text, "rb") as f:
                text = f.read().split(b"\0")[0].decode("latin-1")
        except OSError:
            text = ""
    if p.get("isstring"):
        return text.encode("latin-1")
    out = []
    for tok in [t for t in text.split(" ") if t]:
        h = ""
        for ch in tok[:2]:
            if ch in "0123456789abcdefABCDEF":
                h += ch
            else:
                break
        out.append(int(h, 16) if h else 0)
    return bytes(out)


def build(cfg, seq_idx, first_iter, n_iter, seed_base, literal=False, single_fold=False):
    ip = cfg.get("ip", {})
    proto = {"tcp": 6, "icmp": 1}.get((ip.get("protocol") or "udp").lower(), 17)
    l4len = 20 if proto == 6 else 8
    ttl = ip.get("ttl", {})
    tmin, tmax = ttl.get("min", 64), ttl.get("max", 64)
    idd = ip.get("id", {})
    imin, imax = idd.get("min", 0), idd.get("max", 64000)
    tos = ip.get("tos", 0)
    ipc = ip.get("csum", 1)
    l4c = cfg.get("l4csum", 1)
    eth = cfg.get("eth", {})
    ethhdr = mac(eth.get("dmac")) + mac(eth.get("smac")) + b"\x08\x00"
    daddr = inet_aton(ip["dip"]) or 0
    ranges = [parse_range(r) for r in ip.get("ranges", [])]
    key = "udp" if proto == 17 else "tcp"
    ports = cfg.get(key, {})
    sp_s, dp_s = ports.get("sport", 0), ports.get("dport", 0)
    tcp = cfg.get("tcp", {})
    flags = 0
    for b, n in enumerate(("fin", "syn", "rst", "psh", "ack", "urg", "ece", "cwr")):
        flags |= (tcp.get(n, 0) & 1) << b
    icmp = cfg.get("icmp", {})

    # payload setup (sequence.c:264-374)
    pls = []
    dl0 = []
    ss = seed(seed_base, seq_idx, 0xFFFFFFFFFFFF)
    for i, p in enumerate(cfg.get("payloads", [])):
        ln = p.get("length", {})
        lo, hi = ln.get("min", 0), ln.get("max", 0)
        if p.get("exact") is not None:
            b = exact_bytes(p)
            pls.append(("static", b))
            dl0.append(len(b))
        elif p.get("isstatic") and hi > 0:
            n = rand_num(lo, hi, ss)
            dl = dl0 + [n]
            buf = bytearray(n)
            j = 0
            if literal:
                while j < len(dl) and j < dl[j]:
                    r, ss = rand_r(ss)
                    if j < n:
                        buf[j] = r & 0xFF
                    j += 1
            else:
                for j in range(n):
                    r, ss = rand_r(ss)
                    buf[j] = r & 0xFF
            pls.append(("static", bytes(buf)))
            dl0.append(n)
        elif hi > 0:
            pls.append(("random", (lo, hi)))
            dl0.append(0)
        else:
            pls.append(("static", b""))
            dl0.append(0)
    if not pls:
        pls = [("static", b"")]
        dl0 = [0]

    frames = []
    for k in range(first_iter, first_iter + n_iter):
        s = seed(seed_base, seq_idx, k)
        r0 = rand_r(s)[0]
        t = tmax if tmin == tmax else (r0 % (tmax - tmin + 1) + tmin) & 0xFF
        i_d = imax if imin == imax else (r0 % (imax - imin + 1) + imin) & 0xFFFF
        if ip.get("sip") is not None:
            saddr = inet_aton(ip["sip"]) or 0
        elif ranges:
            rg = ranges[r0 % len(ranges)]
            saddr = 0x7F000001 if rg is None else (rg[0] | (r0 & rg[1]))
        else:
            saddr = 0x7F000001
        prt = 1 + r0 % 65535
        sp = sp_s if sp_s else prt
        dp = dp_s if dp_s else prt
        dl = list(dl0)
        for i, (kind, val) in enumerate(pls):
            if kind == "static":
                payload = val
            else:
                n = rand_num(val[0], val[1], s)
                dl[i] = n
                buf = bytearray(n)
                if literal:
                    j = 0
                    while j < len(dl) and j < dl[j]:
                        r, s = rand_r(s)
                        if j < n:
                            buf[j] = r & 0xFF
                        j += 1
                else:
                    for j in range(n):
                        r, s = rand_r(s)
                        buf[j] = r & 0xFF
                payload = bytes(buf)
            l4tot = l4len + len(payload)
            if proto == 17:
                l4 = struct.pack("!HHHH", sp, dp, l4tot, 0) + payload
            elif proto == 6:
                l4 = struct.pack("!HHIIBBHHH", sp, dp, 0, 0, 0x50, flags, 0, 0, 0) + payload
            else:
                l4 = struct.pack("!BBHI", icmp.get("type", 0), icmp.get("code", 0), 0, 0) + payload
            if l4c:
                if proto == 1:
                    c = csum(l4)
                else:
                    c = csum(struct.pack("!IIBBH", saddr, daddr, 0, proto, l4tot) + l4)
                pos = {17: 6, 6: 16, 1: 2}[proto]
                l4 = l4[:pos] + struct.pack("!H", c) + l4[pos + 2:]
            hdr = struct.pack("!BBHHHBBHII", 0x45, tos, 20 + l4tot, i_d, 0, t, proto, 0, saddr, daddr)
            if ipc:
                c = csum_single(hdr) if single_fold else csum(hdr)
                hdr = hdr[:10] + struct.pack("!H", c) + hdr[12:]
            frames.append(ethhdr + hdr + l4)
    return frames

"""Named subscription sets used by the golden fixtures and parity tests."""
from retina_amd import synth

QUIRKS_SUBS = [
    # overlapping subnets nest (is_child), siblings chain with else-if (is_excl / outcome_eq)
    ("ipv4.src_addr = 10.0.0.0/8 and tcp", ["ZcFrame"], "a_cb"),
    ("ipv4.src_addr = 10.1.0.0/16 and tcp.dst_port = 80", ["ConnRecord"], "b_cb"),
    ("ipv4.src_addr = 10.1.2.0/24", ["Payload", "FilterStr"], "c_cb"),
    ("ipv4.dst_addr = 10.0.0.2 or ipv6.dst_addr = 2001:db8::2", ["ZcFrame", "CoreId"], "d_cb"),
    ("tcp.port in 1000..2000 or udp.port >= 5000", ["ConnRecord"], "e_cb"),
    ("tcp.dst_port < 100 and tcp.dst_port > 20", ["ZcFrame", "FilterStr"], "f_cb"),
    ("tcp.dst_port = 80", ["ZcFrame", "FilterStr"], "g_cb"),
    ("tcp.dst_port = 80", ["ZcFrame", "FilterStr"], "g_cb"),
    ("ipv4.time_to_live >= 64 and udp", ["Payload"], "h_cb"),
    ("ipv6.next_header = 6 and ipv6.hop_limit = 64", ["ZcFrame"], "i_cb"),
    ("tcp.synack = 1 and tcp.data_offset > 5", ["ZcFrame"], "j_cb"),
    ("ipv4.df = 0.0.0.1", ["ZcFrame"], "k_cb"),
    ("ipv4.protocol = 17 and udp.length < 30", ["ZcFrame"], "l_cb"),
    ("ipv6.src_addr != 2001:db8::/32", ["ConnRecord"], "m_cb"),
]

PAYLOAD_SUBS = [
    ("tcp.dst_port = 80", ["Payload"], "p80_cb"),
    ("udp", ["Payload", "FilterStr"], "pudp_cb"),
    ("ipv4 or ipv6", ["ZcFrame"], "any_cb"),
]

PORT_COUNT_SUBS = [("udp", ["ZcFrame", "CoreId"], "udp_cb"), ("tcp", ["ZcFrame", "CoreId"], "tcp_cb"),
                   ("tcp or udp", ["ConnRecord"], "conn_cb")]

# the connection stage (first-packet packet_filter): static-level subscriptions delivered inside
# packet_filter, connection/session-level actions, a streaming subscription, IPv6 prefixes
CONN_SUBS = [
    ("ipv4.src_addr = 10.0.0.0/8 and tcp.dst_port = 80", ["FiveTuple"], "ft_cb"),
    ("tcp.port = 443", ["ConnRecord"], "conn_cb"),
    ("ipv6.dst_addr = 2001:db8::/32 and udp", ["FiveTuple", "FilterStr"], "v6_cb"),
    ("tls", ["TlsHandshake"], "tls_cb"),
    ("tcp.src_port >= 1024 and ipv4.dst_addr != 10.0.0.0/8", ["ConnRecord"], "hi_cb"),
    ("udp.port = 53", ["PktCount", "FiveTuple"], "dns_stream_cb", "packets=1"),
    ("tcp.dst_port = 25", ["ZcFrame"], "smtp_pkt"),
    ("ipv6.src_addr = ::1/128 or ipv4.addr = 192.168.0.0/16", ["FiveTuple"], "local_cb"),
]

MATCH_ALL_SUBS = [("", ["ZcFrame"], "all_cb"), ("", ["ConnRecord"], "conn_cb")]

SETS = {
    "cfg2": synth.CFG2_SPEC,
    "basic": synth.BASIC_SPEC,
    "cfg3": synth.CFG3_SPEC,
    "cfg4": synth.CFG4_SPEC,
    "quirks": synth._toml(QUIRKS_SUBS),
    "payload": synth._toml(PAYLOAD_SUBS),
    "port_count": synth._toml(PORT_COUNT_SUBS),
    "match_all": synth._toml(MATCH_ALL_SUBS),
    "conn": synth._toml(CONN_SUBS),
}

"""Extract the FiveTuples of the reference's end-to-end golden output (run here, where
/root/reference is mounted):

    python tests/golden/make_basic_tuples.py

tests/functionality/basic_test/expected_output_basic.txt is what basic_test (a `#[filter("tls")]`
app, src/main.rs:39-54) prints over traces/small_flows.pcap: a pretty JSON array of {sni,
five_tuple: {orig, resp, proto}, byte_count}, then a "TLS Callback Count" line. The pcap itself is
absent (.MISSING_LARGE_BLOBS), so only the tuples are usable: they pin FiveTuple's orientation
(orig = the first packet's source, conn_id.rs:32-38 / conn_info.rs:33-39) and its serde format
(SocketAddr Display). Writes basic_five_tuples.json: the 60 records' five_tuple objects, in order.
"""
import json
from pathlib import Path

SRC = Path("/root/reference/tests/functionality/basic_test/expected_output_basic.txt")
OUT = Path(__file__).resolve().parent / "basic_five_tuples.json"


def main() -> None:
    text = SRC.read_text()
    records, end = json.JSONDecoder().raw_decode(text)
    assert text[end:].strip() == f"TLS Callback Count: {len(records)}"
    OUT.write_text(json.dumps([r["five_tuple"] for r in records], indent=1) + "\n")
    print(len(records), "tuples ->", OUT)


if __name__ == "__main__":
    main()

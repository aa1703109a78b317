"""Write tests/golden/kat.json — known-answer vectors that pin the oracle.

Nothing here is computed by the oracle or by the product.  Every expected value
is transcribed from one of three sources, named in each vector's "source":

  * SURVEY.md §8a Q1-Q7 — outputs of the reference's own ws.cpp observed in
    the survey container ([probe] entries); the reference itself cannot be
    rebuilt in this round ("Oracle and parity pinning");
  * the reference's tests/test_ws.cpp byte-count expectations;
  * RFC 6455 §5.7 worked examples, for the cases where the reference follows
    the RFC (data frames; receive side of control frames).

Large payloads are described by a generator ("pattern") instead of bytes:
  "zeros:N"      N zero bytes,
  "ramp:N"       bytes i & 0xFF for i in [0, N).

Run:  python tests/golden/make_golden.py
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))

SURVEY_KEY = "d4c3b2a1"      # key bytes _ws_send_mask[0..3] used by the SURVEY probes
RFC_KEY = "37fa213d"         # masking key of RFC 6455 §5.7


def h(s):
    return s.replace(" ", "")


ENCODE = [
    # PrepareSendFrame(opcode, mask, payload, status) with _ws_send_mask = key
    dict(name="q1_pong_unmasked_still_xored", source="SURVEY.md §8a Q1 [probe]",
         opcode=0x8A, mask=False, key=SURVEY_KEY, payload=h("7a"), status=0,
         expect=h("8a 03 d4 c3 c8")),
    dict(name="q2_close_empty_no_status", source="SURVEY.md §8a Q2 [probe]",
         opcode=0x88, mask=True, key=SURVEY_KEY, payload="", status=0,
         expect=h("88 80 d4 c3 b2 a1")),
    dict(name="q4_len126_unmasked", source="SURVEY.md §8a Q4 [probe]",
         opcode=0x82, mask=False, key="00000000", pattern="zeros:126", status=0,
         expect_prefix=h("82 7e 00 7e"), expect_len=130),
    dict(name="q4_len65536_masked_8byte_form", source="SURVEY.md §8a Q4 [probe]",
         opcode=0x82, mask=True, key=SURVEY_KEY, pattern="zeros:65536", status=0,
         expect_prefix=h("82 ff 00 00 00 00 00 01 00 00") + SURVEY_KEY, expect_len=65550),
    dict(name="q2_server_ping_status_prefix", source="SURVEY.md §8a Q2 [probe] (ping 'ab' -> '00 00 61 62')",
         opcode=0x89, mask=False, key="00000000", payload=h("61 62"), status=0,
         expect=h("89 04 00 00 61 62")),
    dict(name="rfc_masked_hello", source="RFC 6455 §5.7",
         opcode=0x81, mask=True, key=RFC_KEY, payload="48656c6c6f", status=0,
         expect=h("81 85 37 fa 21 3d 7f 9f 4d 51 58")),
    dict(name="rfc_unmasked_hello", source="RFC 6455 §5.7",
         opcode=0x81, mask=False, key="00000000", payload="48656c6c6f", status=0,
         expect=h("81 05 48 65 6c 6c 6f")),
    dict(name="rfc_binary_256_unmasked", source="RFC 6455 §5.7",
         opcode=0x82, mask=False, key="00000000", pattern="ramp:256", status=0,
         expect_prefix=h("82 7e 01 00"), expect_len=260, expect_payload_identity=True),
    dict(name="rfc_binary_65536_unmasked", source="RFC 6455 §5.7",
         opcode=0x82, mask=False, key="00000000", pattern="ramp:65536", status=0,
         expect_prefix=h("82 7f 00 00 00 00 00 01 00 00"), expect_len=65546,
         expect_payload_identity=True),
]

DECODE = [
    # Feed `chunks` to PrepareReceiveFrame in order; expect callbacks `events`
    # as [kind, payload_hex, status]; kinds: received / close / ping / pong.
    dict(name="rfc_unmasked_hello", source="RFC 6455 §5.7",
         chunks=[h("81 05 48 65 6c 6c 6f")], events=[["received", "48656c6c6f", 0]]),
    dict(name="rfc_masked_hello", source="RFC 6455 §5.7",
         chunks=[h("81 85 37 fa 21 3d 7f 9f 4d 51 58")], events=[["received", "48656c6c6f", 0]]),
    dict(name="rfc_fragmented_hello", source="RFC 6455 §5.7",
         chunks=[h("01 03 48 65 6c"), h("80 02 6c 6f")], events=[["received", "48656c6c6f", 0]]),
    dict(name="rfc_fragmented_one_read", source="RFC 6455 §5.7 (both frames in one read)",
         chunks=[h("01 03 48 65 6c 80 02 6c 6f")], events=[["received", "48656c6c6f", 0]]),
    dict(name="rfc_unmasked_ping", source="RFC 6455 §5.7",
         chunks=[h("89 05 48 65 6c 6c 6f")], events=[["ping", "48656c6c6f", 0]]),
    dict(name="rfc_masked_pong", source="RFC 6455 §5.7",
         chunks=[h("8a 85 37 fa 21 3d 7f 9f 4d 51 58")], events=[["pong", "48656c6c6f", 0]]),
    dict(name="q5_continuation_concat", source="SURVEY.md §8a Q5 [probe] ('ab' + 'cd' -> one 'abcd')",
         chunks=[h("01 02 61 62"), h("80 02 63 64")], events=[["received", "61626364", 0]]),
]

ROUNDTRIP = [
    # client encodes with key, server session decodes: expected callbacks
    dict(name="q2_client_ping_status_prefix", source="SURVEY.md §8a Q2 [probe]",
         opcode=0x89, mask=True, key=SURVEY_KEY, payload="6162", status=0,
         events=[["ping", "00006162", 0]]),
    dict(name="q6_close_status_text", source="SURVEY.md §8a Q6 [probe] (1001 + 'bye')",
         opcode=0x88, mask=True, key=SURVEY_KEY, payload="627965", status=1001,
         events=[["close", "627965", 1001]]),
    dict(name="test_ws_echo_text", source="reference tests/test_ws.cpp:142 (SendTextAsync('test') -> 4 bytes)",
         opcode=0x81, mask=True, key=SURVEY_KEY, payload="74657374", status=0,
         events=[["received", "74657374", 0]]),
    dict(name="test_ws_multicast_text", source="reference ws_server.h:50 + tests/test_ws.cpp:212 (4 bytes per client)",
         opcode=0x81, mask=False, key="00000000", payload="74657374", status=0,
         events=[["received", "74657374", 0]]),
]

SPLIT = [
    # one masked frame delivered in two reads split at byte offset k;
    # which splits deliver the original payload (Q7 streaming quirk)
    dict(name="q7_masked_10byte_frame", source="SURVEY.md §8a Q7 [probe]",
         opcode=0x82, key=SURVEY_KEY, payload="01020304",
         wrong_at=[1, 3, 4, 5], correct_at=[2, 6, 7, 8, 9]),
    dict(name="q7_masked_300byte_frame_odd_splits", source="SURVEY.md §8a Q7 [probe] (300-B frame, splits 1,3,5,7 wrong)",
         opcode=0x82, key=SURVEY_KEY, pattern="ramp:292",
         wrong_at=[1, 3, 5, 7], correct_at=[]),
]


def main():
    doc = dict(
        comment="Known-answer vectors pinning oracle/ws_oracle.cpp; see make_golden.py for sources.",
        encode=ENCODE, decode=DECODE, roundtrip=ROUNDTRIP, split=SPLIT,
    )
    path = os.path.join(HERE, "kat.json")
    with open(path, "w") as f:
        json.dump(doc, f, indent=1)
    print("wrote", path)


if __name__ == "__main__":
    main()

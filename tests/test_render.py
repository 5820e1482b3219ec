"""The offline Helm renderer (testing/render.py) against Go text/template + Helm semantics, for
every construct the chart uses.  No helm binary exists here, so the chart's rendering is only as
faithful as this subset; these cases pin the behaviour Helm 3 has (expected outputs are Helm's)."""

import pytest

from network_operator_amd.testing.render import render_template as R

CASES = [
    ('a {{- "b" -}} c', {}, "abc"),                                     # trim markers eat whitespace
    ('a {{ "b" }} c', {}, "a b c"),
    ('{{ .Values.n | default 5 }}', {"n": 0}, "5"),                     # sprig default: 0 is empty
    ('{{ .Values.n | default 5 }}', {"n": 3}, "3"),
    ('{{ .Values.f | default false }}', {"f": True}, "true"),           # Go prints bools lower-case
    ('{{ .Values.f }}', {"f": False}, "false"),
    ('{{ .Values.n }}', {"n": 9000}, "9000"),
    ('{{ .Values.missing }}', {}, ""),                                  # Helm strips "<no value>"
    ('{{ .Values.m | toYaml | nindent 2 }}', {"m": {"k": "v", "a": 1}}, "\n  a: 1\n  k: v"),  # sorted keys
    ('{{ .Values.l | toYaml | nindent 4 }}', {"l": ["x", "y"]}, "\n    - x\n    - y"),
    ('{{ if has .Values.mode (list "L2" "L3") }}ok{{ end }}', {"mode": "L3"}, "ok"),
    ('{{ if has .Values.mode (list "L2" "L3") }}ok{{ end }}', {"mode": "L4"}, ""),
    ('{{ if or (lt (int .Values.x) 1500) (gt (int .Values.x) 9000) }}bad{{ end }}', {"x": 9000}, ""),
    ('{{ if or (lt (int .Values.x) 1500) (gt (int .Values.x) 9000) }}bad{{ end }}', {"x": "100"}, "bad"),
    ('{{ quote .Values.s }}', {"s": 'a"b'}, '"a\\"b"'),
    ('{{ .Release.Namespace }}', {}, "ns"),
    ('x\n{{- if .Values.a }}\ny{{- end }}\nz', {"a": True}, "x\ny\nz"),
    ('x\n{{- if .Values.a }}\ny{{- end }}\nz', {"a": False}, "x\nz"),
]


@pytest.mark.parametrize("src,values,want", CASES)
def test_go_template_semantics(src, values, want):
    assert R(src, values, "ns") == want


def test_fail_aborts_the_render():
    with pytest.raises(Exception, match="MTU must be"):
        R('{{- fail "MTU must be between 1500 and 9000" }}', {}, "ns")

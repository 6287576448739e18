"""Chat templates (Jinja2, sandboxed) for /v1/chat/completions.

Compatibility: the reference ships two ConfigMaps, ``phi-chat-template`` and
``opt-chat-template`` (templates/phi-chat-template.yaml:1-24, opt-...:1-24), each with
key ``template.jinja``.  They differ only in the user-turn tag ("Human" / "User"); the
builder below reproduces their template text byte for byte, quirks included: the
``{%- -%}`` whitespace control strips the intended blank lines, so turns are
concatenated with no separator, and the generation prompt opens a new *user* turn.
Those two stay available by name.  The engine's default ("turns") is the corrected form:
turns separated by a blank line and a generation prompt that opens the assistant turn.
Qwen3-style ChatML is also provided.
"""
from __future__ import annotations

import os
from typing import Optional

import jinja2
import jinja2.sandbox


def _legacy_turn_template(user_tag: str) -> str:
    """Exact template text of the reference's phi/opt ConfigMaps (after YAML parsing)."""
    sys_block = (
        "{%- if messages[0]['role'] == 'system' -%}\n"
        "    {%- set system_message = messages[0]['content'] + '\\n\\n' -%}\n"
        "    {%- set messages = messages[1:] -%}\n"
        "{%- else -%}\n"
        "    {%- set system_message = '' -%}\n"
        "{%- endif -%}\n\n"
        "{{- system_message -}}\n"
    )
    turns = "{%- for message in messages -%}\n"
    for i, (role, tag) in enumerate((("user", user_tag), ("assistant", "Assistant"))):
        kw = "if" if i == 0 else "elif"
        turns += (f"    {{%- {kw} message['role'] == '{role}' -%}}\n"
                  f"{tag}: {{{{ message['content'] }}}}\n\n")
    turns += "    {%- endif -%}\n{%- endfor -%}\n"
    gen = f"{{%- if add_generation_prompt -%}}\n{user_tag}: {{% endif %}} "
    return sys_block + turns + gen


TURNS_TEMPLATE = (
    "{%- for message in messages -%}"
    "{%- if message['role'] == 'system' -%}{{ message['content'] + '\\n\\n' }}"
    "{%- elif message['role'] == 'user' -%}{{ 'User: ' + message['content'] + '\\n\\n' }}"
    "{%- elif message['role'] == 'assistant' -%}"
    "{{ 'Assistant: ' + message['content'] + '\\n\\n' }}"
    "{%- endif -%}"
    "{%- endfor -%}"
    "{%- if add_generation_prompt -%}{{ 'Assistant:' }}{%- endif -%}"
)

CHATML_TEMPLATE = (
    "{%- for message in messages -%}"
    "{{ '<|im_start|>' + message['role'] + '\\n' + message['content'] + '<|im_end|>\\n' }}"
    "{%- endfor -%}"
    "{%- if add_generation_prompt -%}{{ '<|im_start|>assistant\\n' }}{%- endif -%}"
)

BUILTIN = {
    "phi": _legacy_turn_template("Human"),
    "opt": _legacy_turn_template("User"),
    "turns": TURNS_TEMPLATE,
    "chatml": CHATML_TEMPLATE,
}
BUILTIN["default"] = BUILTIN["turns"]

_ENV = jinja2.sandbox.ImmutableSandboxedEnvironment(undefined=jinja2.StrictUndefined)


def configmap_name(name: str) -> str:
    return f"{name}-chat-template"


def load_template(spec: Optional[str]) -> str:
    """Resolve a template spec: builtin name, .jinja path, ConfigMap YAML path, or inline."""
    if not spec:
        return BUILTIN["default"]
    if spec in BUILTIN:
        return BUILTIN[spec]
    if spec.endswith("-chat-template") and spec[: -len("-chat-template")] in BUILTIN:
        return BUILTIN[spec[: -len("-chat-template")]]
    if os.path.exists(spec):
        with open(spec) as f:
            text = f.read()
        if spec.endswith((".yaml", ".yml")):
            import yaml

            for doc in yaml.safe_load_all(text):
                if doc and doc.get("kind") == "ConfigMap" and "template.jinja" in doc.get("data", {}):
                    return doc["data"]["template.jinja"]
            raise ValueError(f"{spec}: no ConfigMap with data['template.jinja']")
        return text
    if "{%" in spec or "{{" in spec:
        return spec
    raise ValueError(f"unknown chat template {spec!r}")


def render(messages: list[dict], template: Optional[str] = None,
           add_generation_prompt: bool = True, **extra) -> str:
    tmpl = _ENV.from_string(template if template is not None else BUILTIN["default"])
    msgs = [{"role": m.get("role", "user"), "content": _content_text(m.get("content", ""))}
            for m in messages]
    return tmpl.render(messages=msgs, add_generation_prompt=add_generation_prompt, **extra)


def _content_text(content) -> str:
    if isinstance(content, str):
        return content
    if isinstance(content, list):  # OpenAI content parts
        return "".join(p.get("text", "") for p in content if isinstance(p, dict))
    return str(content)


def configmap_yaml(name: str, template: str, namespace: Optional[str] = None) -> dict:
    meta = {"name": configmap_name(name)}
    if namespace:
        meta["namespace"] = namespace
    return {"apiVersion": "v1", "kind": "ConfigMap", "metadata": meta,
            "data": {"template.jinja": template}}


def configmap_text(name: str) -> str:
    """The ConfigMap manifest of builtin template `name` as YAML text in the reference's
    layout (templates/<name>-chat-template.yaml: a `|-` block scalar indented 4 spaces) --
    for phi / opt byte-identical to the reference files (pinned by tests/test_provisioning)."""
    body = "\n".join(("    " + ln) if ln else "" for ln in BUILTIN[name].split("\n"))
    return ("apiVersion: v1\nkind: ConfigMap\nmetadata:\n"
            f"  name: {configmap_name(name)}\ndata:\n  template.jinja: |-\n{body}")


def main(argv=None) -> int:
    """python -m aws_k8s_ansible_provisioner_amd.utils.chat_template --write-configmaps DIR
    writes <name>-chat-template.yaml for the reference-compatible phi / opt templates (and
    the corrected default) so `kubectl apply -f DIR` installs them as the reference did."""
    import argparse

    ap = argparse.ArgumentParser()
    ap.add_argument("--write-configmaps", metavar="DIR", required=True)
    ap.add_argument("--names", default="phi,opt,default")
    a = ap.parse_args(argv)
    os.makedirs(a.write_configmaps, exist_ok=True)
    for n in a.names.split(","):
        path = os.path.join(a.write_configmaps, f"{configmap_name(n)}.yaml")
        with open(path, "w") as f:
            f.write(configmap_text(n))
        print(path)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())

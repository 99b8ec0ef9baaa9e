#!/usr/bin/env python3
"""Mechanical TypeScript type-erasure for the golden-fixture generator.

TEST INFRASTRUCTURE ONLY.  This reads reference ``.ts`` files from
``/root/reference/src`` at generation time and writes plain CommonJS into a
scratch directory under ``/tmp`` (never into this repository).  It removes
*only* what TypeScript itself erases -- type annotations, ``type`` aliases,
``interface`` blocks, ``as`` casts, ``private`` modifiers and bodiless class
field declarations -- and rewrites ES ``import``/``export`` into
``require``/``module.exports`` so Node 12 (the only Node in the image) can run
the result.  ``a ?? b`` (not parsed by Node 12) is lowered to
``__nc(a, b)`` with the exact nullish semantics.  No runtime expression of the
reference is altered.

After stripping, the token stream of the output is checked to be a
subsequence of the input token stream (plus the import/export/``??``
rewrites), so nothing but type syntax can have been dropped.
"""
import re
import sys

PUNCT = [
    '>>>=', '...', '===', '!==', '**=', '<<=', '>>=', '>>>', '&&=', '||=', '??=',
    '=>', '==', '!=', '<=', '>=', '&&', '||', '??', '?.', '++', '--', '+=', '-=', '*=',
    '/=', '%=', '&=', '|=', '^=', '<<', '>>', '**',
]


class Tok:
    __slots__ = ('kind', 'text')

    def __init__(self, kind, text):
        self.kind = kind
        self.text = text

    def __repr__(self):
        return f'{self.kind}:{self.text!r}'


def tokenize(src):
    toks = []
    i = 0
    n = len(src)
    prev_sig = None  # last significant token (for regex detection)
    while i < n:
        c = src[i]
        if c in ' \t\r\n':
            j = i
            while j < n and src[j] in ' \t\r\n':
                j += 1
            toks.append(Tok('ws', src[i:j]))
            i = j
            continue
        if src.startswith('//', i):
            j = src.find('\n', i)
            j = n if j < 0 else j
            toks.append(Tok('comment', src[i:j]))
            i = j
            continue
        if src.startswith('/*', i):
            j = src.find('*/', i + 2) + 2
            toks.append(Tok('comment', src[i:j]))
            i = j
            continue
        if c in '\'"':
            j = i + 1
            while src[j] != c:
                j += 2 if src[j] == '\\' else 1
            toks.append(Tok('str', src[i:j + 1]))
            prev_sig = toks[-1]
            i = j + 1
            continue
        if c == '`':
            # template literal with nested ${ ... } (braces balanced, strings inside skipped)
            j = i + 1
            while True:
                if src[j] == '\\':
                    j += 2
                    continue
                if src[j] == '`':
                    break
                if src.startswith('${', j):
                    depth = 1
                    j += 2
                    while depth:
                        if src[j] in '\'"':
                            q = src[j]
                            j += 1
                            while src[j] != q:
                                j += 2 if src[j] == '\\' else 1
                        elif src[j] == '{':
                            depth += 1
                        elif src[j] == '}':
                            depth -= 1
                        j += 1
                    continue
                j += 1
            toks.append(Tok('str', src[i:j + 1]))
            prev_sig = toks[-1]
            i = j + 1
            continue
        if c == '/' and (prev_sig is None or (prev_sig.kind == 'punct' and prev_sig.text not in (')', ']', '}'))
                         or (prev_sig.kind == 'ident' and prev_sig.text in ('return', 'typeof', 'case'))):
            # regex literal
            j = i + 1
            in_cls = False
            while True:
                if src[j] == '\\':
                    j += 2
                    continue
                if src[j] == '[':
                    in_cls = True
                elif src[j] == ']':
                    in_cls = False
                elif src[j] == '/' and not in_cls:
                    break
                j += 1
            j += 1
            while j < n and src[j].isalpha():
                j += 1
            toks.append(Tok('regex', src[i:j]))
            prev_sig = toks[-1]
            i = j
            continue
        m = re.match(r'[A-Za-z_$][\w$]*', src[i:])
        if m:
            toks.append(Tok('ident', m.group(0)))
            prev_sig = toks[-1]
            i += len(m.group(0))
            continue
        m = re.match(r'(0[xX][0-9a-fA-F]+|\d+\.?\d*(?:[eE][+-]?\d+)?|\.\d+(?:[eE][+-]?\d+)?)', src[i:])
        if m:
            toks.append(Tok('num', m.group(0)))
            prev_sig = toks[-1]
            i += len(m.group(0))
            continue
        for p in PUNCT:
            if src.startswith(p, i):
                toks.append(Tok('punct', p))
                i += len(p)
                break
        else:
            toks.append(Tok('punct', c))
            i += 1
        prev_sig = toks[-1]
    return toks


OPEN = {'(': ')', '[': ']', '{': '}'}


class Stripper:
    def __init__(self, toks):
        self.t = toks
        self.sig = [k for k, tk in enumerate(toks) if tk.kind not in ('ws', 'comment')]
        self.pos = {k: s for s, k in enumerate(self.sig)}
        self.drop = set()
        self.type_names = set()
        self.match = {}
        stack = []
        for k in self.sig:
            tx = toks[k].text
            if toks[k].kind == 'punct' and tx in OPEN:
                stack.append(k)
            elif toks[k].kind == 'punct' and tx in (')', ']', '}'):
                o = stack.pop()
                self.match[o] = k
                self.match[k] = o

    # --- helpers over significant tokens -------------------------------------
    def s(self, si):
        return self.t[self.sig[si]] if 0 <= si < len(self.sig) else Tok('eof', '')

    def txt(self, si):
        return self.s(si).text

    def msi(self, si):
        """significant index of the bracket matching the one at si"""
        return self.pos[self.match[self.sig[si]]]

    def drop_range(self, a, b):
        """drop significant tokens a..b-1 and every ws/comment token between them"""
        if a >= b:
            return
        lo = self.sig[a]
        hi = self.sig[b - 1]
        for k in range(lo, hi + 1):
            self.drop.add(k)

    # --- type expression parser (returns significant index after the type) ----
    def parse_type(self, si):
        si = self.parse_inter(si)
        while self.txt(si) == '|':
            si = self.parse_inter(si + 1)
        return si

    def parse_inter(self, si):
        si = self.parse_postfix(si)
        while self.txt(si) == '&':
            si = self.parse_postfix(si + 1)
        return si

    def parse_postfix(self, si):
        si = self.parse_primary(si)
        while self.txt(si) == '[' and self.txt(si + 1) == ']':
            si += 2
        return si

    def parse_primary(self, si):
        tk = self.s(si)
        if tk.text == 'new':
            return self.parse_primary(si + 1)
        if tk.text == '(':
            end = self.msi(si)
            if self.txt(end + 1) == '=>':
                return self.parse_type(end + 2)
            return end + 1
        if tk.text in ('{', '['):
            return self.msi(si) + 1
        if tk.kind in ('str', 'num'):
            return si + 1
        if tk.kind == 'ident':
            si += 1
            while self.txt(si) == '.' and self.s(si + 1).kind == 'ident':
                si += 2
            if self.txt(si) == '<':
                depth = 0
                while True:
                    x = self.txt(si)
                    if x == '<':
                        depth += 1
                    elif x == '>':
                        depth -= 1
                    elif x == '>>':
                        depth -= 2
                    si += 1
                    if depth <= 0:
                        break
            return si
        raise SyntaxError(f'cannot parse type at {tk!r}')

    # --- context detection -----------------------------------------------------
    def is_param_list(self, si, class_body_open):
        """si indexes a '(' ; decide whether it opens a function parameter list"""
        prev = self.s(si - 1)
        end = self.msi(si)
        nxt = self.txt(end + 1)
        if nxt == '=>':
            return True
        if nxt == ':':
            try:
                after = self.parse_type(end + 2)
            except (SyntaxError, KeyError):
                after = None
            if after is not None and self.txt(after) in ('=>', '{'):
                if self.txt(after) == '=>' or prev.text == 'function' or self.s(si - 2).text == 'function' \
                        or class_body_open:
                    return True
        if prev.kind == 'ident' and self.s(si - 2).text == 'function':
            return True
        if prev.text == 'function':
            return True
        if class_body_open and prev.kind == 'ident' and nxt in ('{', ':'):
            return True
        return False

    def run(self):
        sig = self.sig
        n = len(sig)
        # class bodies: the '{' after `class Name [extends X]`
        class_bodies = set()
        for si in range(n):
            if self.txt(si) == 'class':
                j = si + 1
                while self.txt(j) != '{':
                    j += 1
                class_bodies.add(j)
        # depth tracking to know the innermost open bracket for each token
        encl = [None] * n
        stack = []
        for si in range(n):
            encl[si] = stack[-1] if stack else None
            x = self.txt(si)
            if self.s(si).kind == 'punct' and x in OPEN:
                stack.append(si)
            elif self.s(si).kind == 'punct' and x in (')', ']', '}'):
                stack.pop()
        param_lists = set()
        for si in range(n):
            if self.txt(si) == '(' and self.s(si).kind == 'punct':
                in_class = encl[si] in class_bodies
                if self.is_param_list(si, in_class):
                    param_lists.add(si)

        si = 0
        while si < n:
            tk = self.s(si)
            x = tk.text
            at_top = encl[si] is None
            # type alias
            if x == 'type' and tk.kind == 'ident' and at_top and self.s(si + 1).kind == 'ident' and self.txt(si + 2) == '=':
                self.type_names.add(self.txt(si + 1))
                j = si + 3
                while not (self.txt(j) == ';' and encl[j] is None):
                    j += 1
                self.drop_range(si, j + 1)
                si = j + 1
                continue
            if x == 'interface' and at_top and self.s(si + 1).kind == 'ident':
                self.type_names.add(self.txt(si + 1))
                j = si + 2
                while self.txt(j) != '{':
                    j += 1
                e = self.msi(j)
                self.drop_range(si, e + 1)
                si = e + 1
                continue
            # catch (e: T)
            if x == 'catch' and self.txt(si + 1) == '(' and self.s(si + 2).kind == 'ident' and self.txt(si + 3) == ':':
                e = self.parse_type(si + 4)
                self.drop_range(si + 3, e)
                si = e
                continue
            # class heritage `implements A, B`
            if x == 'implements' and tk.kind == 'ident':
                j = si + 1
                while self.txt(j) != '{':
                    j += 1
                self.drop_range(si, j)
                si = j
                continue
            if x == 'private' and tk.kind == 'ident' and encl[si] in class_bodies:
                self.drop_range(si, si + 1)
                si += 1
                continue
            # `expr as Type`
            if x == 'as' and tk.kind == 'ident' and encl[si] is not None and self.s(si - 1).kind in ('ident', 'punct', 'num'):
                if self.s(si - 1).text not in ('import', '{', ','):
                    e = self.parse_type(si + 1)
                    self.drop_range(si, e)
                    si = e
                    continue
            # variable declaration annotation
            if x in ('let', 'const', 'var') and self.s(si + 1).kind == 'ident' and self.txt(si + 2) == ':':
                e = self.parse_type(si + 3)
                self.drop_range(si + 2, e)
                si = e
                continue
            # class field: IDENT[?]: Type [= init];   (at class body level)
            if encl[si] in class_bodies and tk.kind == 'ident' and self.txt(si - 1) in ('{', ';', '}') \
                    and (self.txt(si + 1) == ':' or (self.txt(si + 1) == '?' and self.txt(si + 2) == ':')):
                c = si + 1 if self.txt(si + 1) == ':' else si + 2
                e = self.parse_type(c + 1)
                if self.txt(e) == ';':
                    if x == 'static':
                        raise SyntaxError('unexpected static field form')
                    self.drop_range(si, e + 1)  # bodiless declaration: erased
                else:
                    self.drop_range(si + 1, e)
                si = e
                continue
            # parameter annotations
            if x == '(' and si in param_lists:
                end = self.msi(si)
                j = si + 1
                while j < end:
                    if encl[j] == si and self.s(j).kind == 'ident' and self.txt(j - 1) in ('(', ','):
                        c = j + 1
                        if self.txt(c) == '?' and self.txt(c + 1) == ':':
                            self.drop_range(c, c + 1)
                            c += 1
                        if self.txt(c) == ':':
                            e = self.parse_type(c + 1)
                            self.drop_range(c, e)
                            j = e
                            continue
                    j += 1
                # return type
                if self.txt(end + 1) == ':':
                    e = self.parse_type(end + 2)
                    self.drop_range(end + 1, e)
                si += 1
                continue
            si += 1
        return self

    def emit(self):
        return ''.join(tk.text for k, tk in enumerate(self.t) if k not in self.drop)


def lower_modules(src, resolver):
    """ES import/export -> CommonJS, `??` -> __nc()."""
    out = []
    for line in src.split('\n'):
        m = re.match(r"^import\s+\{([^}]*)\}\s+from\s+'([^']+)';\s*$", line)
        if m:
            names = [x.strip() for x in m.group(1).split(',') if x.strip()]
            names = [nm.replace(' as ', ': ') for nm in names]
            out.append(f"const {{ {', '.join(names)} }} = require({resolver(m.group(2))!r});")
            continue
        m = re.match(r"^import\s+(\w+)\s+from\s+'([^']+)';\s*$", line)
        if m:
            out.append(f"const {m.group(1)} = (function (m) {{ return m && m.__esModule ? m.default : (m && m.default) || m; }})(require({resolver(m.group(2))!r}));")
            continue
        m = re.match(r'^export\s+\{([^}]*)\};\s*$', line)
        if m:
            names = [x.strip() for x in m.group(1).split(',') if x.strip()]
            out.append(f"module.exports = {{ {', '.join(names)} }};")
            continue
        out.append(line)
    return '\n'.join(out)


def lower_nullish(src):
    """Rewrite `A ?? B` (Node 12 cannot parse it) into `__nc(A, B)`.

    Operands are delimited at bracket depth 0 of the enclosing expression by
    = , ( ) ; : return and newlines, which covers every site in the files used.
    """
    toks = tokenize(src)
    while True:
        idx = next((k for k, tk in enumerate(toks) if tk.kind == 'punct' and tk.text == '??'), None)
        if idx is None:
            break
        # left operand
        depth = 0
        a = idx - 1
        while a >= 0:
            tk = toks[a]
            if tk.kind == 'punct' and tk.text in (')', ']', '}'):
                depth += 1
            elif tk.kind == 'punct' and tk.text in ('(', '[', '{'):
                if depth == 0:
                    break
                depth -= 1
            elif depth == 0 and ((tk.kind == 'punct' and tk.text in ('=', ',', ';', ':', '?')) or
                                 (tk.kind == 'ident' and tk.text == 'return')):
                break
            a -= 1
        # right operand
        depth = 0
        b = idx + 1
        while b < len(toks):
            tk = toks[b]
            if tk.kind == 'punct' and tk.text in ('(', '[', '{'):
                depth += 1
            elif tk.kind == 'punct' and tk.text in (')', ']', '}'):
                if depth == 0:
                    break
                depth -= 1
            elif depth == 0 and tk.kind == 'punct' and tk.text in (',', ';'):
                break
            b += 1
        left = ''.join(tk.text for tk in toks[a + 1:idx]).strip()
        right = ''.join(tk.text for tk in toks[idx + 1:b]).strip()
        lead = ' ' if toks[a + 1].kind == 'ws' else ''
        new = tokenize(f'{lead}__nc({left}, {right})')
        toks = toks[:a + 1] + new + toks[b:]
    return ''.join(tk.text for tk in toks)


def check_subsequence(orig, stripped):
    """Every significant token of `stripped` (outside rewritten import/export/??
    lines) must appear, in order, in `orig`."""
    o = [tk.text for tk in tokenize(orig) if tk.kind not in ('ws', 'comment')]
    s = [tk.text for tk in tokenize(stripped) if tk.kind not in ('ws', 'comment')]
    j = 0
    for x in s:
        while j < len(o) and o[j] != x:
            j += 1
        if j == len(o):
            return False
        j += 1
    return True


def strip(src):
    st = Stripper(tokenize(src)).run()
    out = st.emit()
    # type-only names cannot be exported at runtime
    def fix_export(m):
        names = [x.strip() for x in m.group(1).split(',') if x.strip() and x.strip() not in st.type_names]
        return 'export { ' + ', '.join(names) + ' };'
    out = re.sub(r'^export\s+\{([^}]*)\};', fix_export, out, flags=re.M)
    if not check_subsequence(src, out):
        raise AssertionError('type erasure removed a non-type token')
    return out


if __name__ == '__main__':
    print(strip(open(sys.argv[1]).read()))

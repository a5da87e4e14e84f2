'use strict';
// Minimal XML reader producing xml-js's "compact" shape (xml2js(text, {compact: true})),
// the form src/index.ts:30-113 walks: attributes under `_attributes`, children grouped by
// tag name (one child -> object, several -> array, document order within a tag).
// Supports what scene files use: prolog, comments, CDATA-free elements, quoted attributes.

function decode(s) {
    return s.replace(/&lt;/g, '<').replace(/&gt;/g, '>').replace(/&quot;/g, '"').replace(/&apos;/g, "'")
        .replace(/&#(\d+);/g, (_, d) => String.fromCharCode(parseInt(d, 10))).replace(/&amp;/g, '&');
}

function xml2js(text) {
    let i = 0;
    const n = text.length;
    const root = {};
    const stack = [root];
    const err = (m) => { throw Error(`XML parse error at ${i}: ${m}`); };
    const add = (parent, name, node) => {
        if (!(name in parent)) parent[name] = node;
        else if (Array.isArray(parent[name])) parent[name].push(node);
        else parent[name] = [parent[name], node];
    };
    while (i < n) {
        const lt = text.indexOf('<', i);
        if (lt === -1) break;
        const txt = text.slice(i, lt).trim();
        if (txt.length && stack.length > 1) {
            const top = stack[stack.length - 1];
            top._text = (top._text || '') + decode(txt);
        }
        i = lt;
        if (text.startsWith('<!--', i)) { const e = text.indexOf('-->', i); if (e < 0) err('unterminated comment'); i = e + 3; continue; }
        if (text.startsWith('<?', i)) { const e = text.indexOf('?>', i); if (e < 0) err('unterminated prolog'); i = e + 2; continue; }
        if (text.startsWith('<!', i)) { const e = text.indexOf('>', i); if (e < 0) err('unterminated declaration'); i = e + 1; continue; }
        if (text.startsWith('</', i)) {
            const e = text.indexOf('>', i);
            if (e < 0) err('unterminated end tag');
            if (stack.length <= 1) err('unbalanced end tag');
            stack.pop();
            i = e + 1;
            continue;
        }
        const m = /^<([A-Za-z_][\w.\-:]*)/.exec(text.slice(i, i + 256));
        if (!m) err('bad tag');
        const name = m[1];
        i += m[0].length;
        const node = {};
        const attrs = {};
        let has_attrs = false;
        for (;;) {
            while (i < n && /\s/.test(text[i])) i++;
            if (text[i] === '/' && text[i + 1] === '>') { i += 2; add(stack[stack.length - 1], name, finish()); break; }
            if (text[i] === '>') { i += 1; add(stack[stack.length - 1], name, finish()); stack.push(node); break; }
            const am = /^([A-Za-z_][\w.\-:]*)\s*=\s*("([^"]*)"|'([^']*)')/.exec(text.slice(i, i + 4096));
            if (!am) err(`bad attribute in <${name}>`);
            attrs[am[1]] = decode(am[3] !== undefined ? am[3] : am[4]);
            has_attrs = true;
            i += am[0].length;
        }
        function finish() { if (has_attrs) node._attributes = attrs; return node; }
    }
    if (stack.length !== 1) throw Error('XML parse error: unclosed element');
    return root;
}

module.exports = { xml2js };

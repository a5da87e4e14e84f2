'use strict';
// Loads the N-API addon (lib/pt_node.node, linked against lib/libpt_hip.so).
// No JS fallback: rendering without the HIP library is an error.
const path = require('path');
let addon = null;
function load() {
    if (addon) return addon;
    const file = process.env.PT_NODE_ADDON || path.join(__dirname, '..', '..', 'lib', 'pt_node.node');
    addon = require(file);
    return addon;
}
module.exports = { load };

'use strict';
// INI scene config -> IniFileScene.  Mirrors src/ts-util/parse-ini.ts:9-55.

/** parse-ini.ts:9-33 */
function parse_ini_file(raw_file) {
    const category_groups = {};
    let current_group = {};
    for (const line of raw_file.split('\n')) {
        if (line[0] === '[') {
            const m = line.match(/(?<=\[).+?(?=\])/);
            const name = m ? m[0].trim() : '';
            category_groups[name] = {};
            current_group = category_groups[name];
        } else {
            if (line.indexOf('=') === -1) continue;
            const field_name = line.match(/(?:(?!=).)*/);
            const field_data = line.match(/(?<==).*/);
            const name = field_name ? field_name[0].trim() : '';
            const data = field_data ? field_data[0].trim() : '';
            current_group[name] = data;
        }
    }
    return category_groups;
}

/** parse-ini.ts:35-55 */
function ini_file_to_ini_scene(file) {
    try {
        return {
            IO: { output: file['IO']['output'], scene: file['IO']['scene'] },
            Settings: {
                directLightingOnly: file['Settings']['directLightingOnly'] === 'true',
                imageHeight: parseInt(file['Settings']['imageHeight']),
                imageWidth: parseInt(file['Settings']['imageWidth']),
                numDirectLightingSamples: parseInt(file['Settings']['numDirectLightingSamples']),
                pathContinuationProb: parseFloat(file['Settings']['pathContinuationProb']),
                samplesPerPixel: parseInt(file['Settings']['samplesPerPixel']),
            },
        };
    } catch (e) {
        throw Error('Error in ini file to ini scene file conversion');
    }
}

module.exports = { parse_ini_file, ini_file_to_ini_scene };
